"""GPU: the end-to-end demo (encoder + Tacotron on PyTorch-ROCm, MI355X vocoder) runs, and the
Tacotron on the GPU tracks the reference fixture (float tolerance: GPU GEMMs reorder sums)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO
from test_e2e import G, run_tacotron

pytestmark = pytest.mark.gpu


def test_tacotron_on_gpu_tracks_reference():
    mel, lin, attn, _ = run_tacotron('cuda')
    assert lin.shape == G['linear'].shape
    # 60 autoregressive decoder steps in fp32 with reordered GPU sums
    assert np.abs(lin - G['linear']).max() < 2e-3
    assert np.abs(attn - G['attn']).max() < 2e-3


def test_demo_cli_end_to_end():
    demo = os.path.join(REPO, 'real-time-voice-cloning_amd', 'demo_cli.py')
    out = subprocess.run([sys.executable, demo, '--random-weights', '0', '--utterances', '3',
                          '--max-frames', '80', '--seed', '1'],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith('{')][-1]
    r = json.loads(line)
    assert r['utterances'] == 3 and len(r['mel_frames']) == 3
    assert r['audio_seconds'] == pytest.approx(3 * 79 * 200 / 16000, abs=1e-3)
    assert r['vocoder_engine'] == 'persist'
