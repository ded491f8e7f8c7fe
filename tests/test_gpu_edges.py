"""GPU edge cases of the vocoder path beyond the golden fixtures, every row against the oracle
restatement (``oracle/wavernn_oracle.py``, pinned by tests/test_oracle_golden.py):

* the demo's own fold geometry (``gen_target`` 200 / ``gen_overlap`` 50 at hop 200, the
  ``hparams`` the reference ships for inference) on both engines;
* ragged multi-utterance batches (different mel lengths -> different fold counts per utterance,
  one batch of rows; the reference vocodes them one by one, ``vocoder/inference.py:40-64``);
* a one-frame mel (the shortest input ``fold_with_overlap`` accepts): the rows match the oracle,
  and ``generate`` fails like the reference's (``fatchord_version.py:253-255`` multiplies the
  last 20 hops by a 20-hop fade; a wave shorter than that raises numpy's broadcast ValueError);
* unbatched unequal lengths, which have no single row length and must be refused.

Bar as tests/test_gpu_parity.py: RAW labels bit-exact.
"""
import numpy as np
import pytest

from conftest import golden_case
from test_gpu_parity import first_divergence, make_model

pytestmark = pytest.mark.gpu


def _oracle_rows(sd, hp, meta, mel_scaled, target, overlap, batched=True, stream=0):
    from oracle.wavernn_oracle import oracle_infer_waveform
    return oracle_infer_waveform(sd, hp, meta['model_type'], mel_scaled, target=target,
                                 overlap=overlap, seed=meta['noise_seed'], stream=stream,
                                 batched=batched, post=False)['labels']


def _device_rows(m, meta, mels, batched, target, overlap):
    import torch
    from wavernn_amd.hparams import sp
    dev = [torch.from_numpy((x / sp.max_abs_value).astype(np.float32)).cuda() for x in mels]
    m.set_seed(meta['noise_seed'])
    lab, roff, S = m.generate_batch_device(dev, batched, target, overlap)
    return lab.cpu().numpy(), roff, S


@pytest.mark.parametrize('engine', ['chain', 'persist'])
def test_demo_fold_geometry_bit_exact(engine):
    """gen_target 200 / overlap 50: 300 steps per row, 17 rows for a 21-frame mel."""
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, hp, sd = make_model(meta)
    m.set_engine(engine)
    m.set_seed(meta['noise_seed'])
    mel = synth_mel(21, 31)
    m.generate(mel[None] / sp.max_abs_value, True, 200, 50, hp.mu_law, sp.preemphasize,
               progress_callback=lambda *a: None)
    assert m.last_engine() == engine
    ref = _oracle_rows(sd, hp, meta, mel, 200, 50)
    assert m.last_labels.shape == ref.shape
    assert np.array_equal(m.last_labels, ref), first_divergence(m.last_labels, ref)


@pytest.mark.parametrize('engine', ['chain', 'persist'])
@pytest.mark.parametrize('case', ['fatchord_raw9_tiny', 'runtimeracer_raw9_tiny',
                                  'geneing_bits10_tiny'])
def test_ragged_utterances_one_batch(case, engine):
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case(case)
    m, hp, sd = make_model(meta)
    m.set_engine(engine)
    lens = [3, 11, 24, 37]
    mels = [synth_mel(T, 300 + u) for u, T in enumerate(lens)]
    lab, roff, S = _device_rows(m, meta, mels, True, meta['target'], meta['overlap'])
    assert m.last_engine() == engine
    assert len(set(np.diff(roff).tolist())) > 1, 'lengths should give different fold counts'
    for u in range(len(lens)):
        ref = _oracle_rows(sd, hp, meta, mels[u], meta['target'], meta['overlap'], stream=u)
        got = lab[roff[u]:roff[u + 1]]
        assert got.shape == ref.shape
        assert np.array_equal(got, ref), f'utt {u}: {first_divergence(got, ref)}'


@pytest.mark.parametrize('batched', [True, False])
def test_single_frame_mel(batched):
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, hp, sd = make_model(meta)
    mel = synth_mel(1, 5)
    lab, roff, S = _device_rows(m, meta, [mel], batched, meta['target'], meta['overlap'])
    ref = _oracle_rows(sd, hp, meta, mel, meta['target'], meta['overlap'], batched=batched)
    assert lab.shape == ref.shape and np.array_equal(lab, ref)
    with pytest.raises(ValueError):  # same failure as the reference's tail fade
        m.generate(mel[None] / sp.max_abs_value, batched, meta['target'], meta['overlap'],
                   hp.mu_law, sp.preemphasize, progress_callback=lambda *a: None)


def test_unbatched_unequal_lengths_refused():
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, hp, sd = make_model(meta)
    with pytest.raises((ValueError, RuntimeError)):
        _device_rows(m, meta, [synth_mel(4, 7), synth_mel(6, 8)], False, meta['target'],
                     meta['overlap'])


@pytest.mark.parametrize('n_utts', [4, 6])
def test_fatchord_10bit_row_groups_match_oracle(n_utts):
    """10-bit fatchord (32 classes per slot, fc3 rows held in registers) at 20 / 30 fold rows:
    the 3- and 4-rows-per-group variants the launch-cost choice takes, every row against the
    oracle."""
    from wavernn_amd.synth import synth_mel
    meta = dict(golden_case('fatchord_raw9_sharp_tiny')[0])
    meta['bits'] = 10
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    mels = [synth_mel(meta['n_frames'], 400 + u) for u in range(n_utts)]
    lab, roff, S = _device_rows(m, meta, mels, True, meta['target'], meta['overlap'])
    assert m.last_engine() == 'persist'
    for u in range(n_utts):
        ref = _oracle_rows(sd, hp, meta, mels[u], meta['target'], meta['overlap'], stream=u)
        got = lab[roff[u]:roff[u + 1]]
        assert np.array_equal(got, ref), f'utt {u}: {first_divergence(got, ref)}'
