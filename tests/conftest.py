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


def golden_meta(regime='bit-exact'):
    """Fixtures by parity regime: 'bit-exact' (every case whose labels a correct fp32
    implementation must reproduce), 'divergence-onset' (the chaotic trained-like case, see
    tests/golden/gen_golden.py), or None for all."""
    with open(os.path.join(GOLDEN, 'golden_meta.json')) as f:
        return {k: v for k, v in json.load(f).items() if not k.startswith('_')
                and (regime is None or v.get('regime', 'bit-exact') == regime)}


def golden_case(name):
    return golden_meta(None)[name], dict(np.load(os.path.join(GOLDEN, name + '.npz')))


def state_dict_of(meta):
    """The fixture's seeded weights (synth_state_dict with the case's statistics knobs)."""
    from wavernn_amd.synth import synth_state_dict
    sd = synth_state_dict(hparams_of(meta), meta['model_type'], seed=meta['weight_seed'],
                          logit_scale=meta['logit_scale'], gru_scale=meta.get('gru_scale', 1.0),
                          fc_scale=meta.get('fc_scale', 1.0))
    if meta.get('prune'):  # pruned checkpoints: the reference Pruner's masks (wavernn_amd.prune)
        from wavernn_amd.prune import prune_state_dict
        sd = prune_state_dict(sd, meta['model_type'], z=meta['prune'], group=4)
    return sd


def wave_equal(wav, gold):
    """Bit equality with the reference's f64 waveform, stored whole or as its SHA-256 (the
    full-size trained-like fixtures)."""
    if 'wav' in gold:
        return wav.shape == gold['wav'].shape and np.array_equal(wav, gold['wav'])
    import hashlib
    return (len(wav) == int(gold['wav_len']) and wav.dtype == np.float64 and
            hashlib.sha256(np.ascontiguousarray(wav).tobytes()).digest() == gold['wav_sha256'].tobytes())


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
