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


@pytest.mark.parametrize('n_utts', [3, 8])
def test_demo_cli_end_to_end(n_utts, tmp_path):
    """The demo at 3 utterances and at the configs[4] shape (8 utterances, one GPU here), and the
    vocoder's part of it against the oracle: utterance 0's Tacotron mel as the vocoder saw it,
    its fold-row labels and waveform, re-run on the host oracle with the same weights, seed and
    noise stream -- labels and f64 waveform bit-exact (BASELINE north_star, 9/10-bit RAW)."""
    demo = os.path.join(REPO, 'real-time-voice-cloning_amd', 'demo_cli.py')
    dump = str(tmp_path / 'utt0.npz')
    out = subprocess.run([sys.executable, demo, '--random-weights', '0', '--utterances', str(n_utts),
                          '--max-frames', '80', '--seed', '1', '--dump', dump],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith('{')][-1]
    r = json.loads(line)
    assert r['utterances'] == n_utts and len(r['mel_frames']) == n_utts
    assert r['audio_seconds'] == pytest.approx(n_utts * 79 * 200 / 16000, abs=1e-3)
    assert r['vocoder_engine'] == 'persist'
    # vocoder parity inside the end-to-end run
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.base import hparams_for
    from wavernn_amd.synth import synth_state_dict
    d = np.load(dump)
    mt = str(d['model_type'])
    hp = hparams_for(mt)
    sd = synth_state_dict(hp, mt, seed=int(d['weights_seed']))
    o = oracle_infer_waveform(sd, hp, mt, d['mel'], normalize=False, batched=True,
                              target=hp.gen_target, overlap=hp.gen_overlap, seed=int(d['seed']),
                              stream=int(d['stream']))
    assert d['rows'].shape == o['labels'].shape
    assert np.array_equal(d['rows'], o['labels']), \
        f"first divergence {np.argwhere(d['rows'] != o['labels'])[:1].tolist()}"
    assert np.array_equal(d['wav'], o['wav'])
