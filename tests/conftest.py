import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'real-time-voice-cloning_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


def golden_meta():
    with open(os.path.join(GOLDEN, 'golden_meta.json')) as f:
        return {k: v for k, v in json.load(f).items() if not k.startswith('_')}


def golden_case(name):
    return golden_meta()[name], dict(np.load(os.path.join(GOLDEN, name + '.npz')))


def is_continuous(meta):
    """Float samples (MOL, geneing 'RAW' Beta) rather than categorical labels."""
    return meta['mode'] == 'MOL' or (meta['model_type'] == 'geneing-wavernn' and meta['mode'] == 'RAW')


def hparams_of(meta):
    from wavernn_amd.hparams import wavernn_fatchord, wavernn_geneing, wavernn_runtimeracer
    base = {'fatchord-wavernn': wavernn_fatchord, 'geneing-wavernn': wavernn_geneing,
            'runtimeracer-wavernn': wavernn_runtimeracer}[meta['model_type']]
    return base.copy(bits=meta['bits'], mode=meta['mode'])


@pytest.fixture(scope='session')
def gpu_available():
    import torch
    return torch.cuda.is_available()
