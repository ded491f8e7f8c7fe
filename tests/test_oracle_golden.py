"""Pins the oracle: the torch-CPU restatement reproduces, bit for bit, the outputs the REAL
reference generate() produced (tests/golden/*.npz, written by tests/golden/gen_golden.py in the
survey container with the reference imported from /root/reference). CPU only.

The full-size trained-like fixtures (217,800 / 270,000 draws) are checked on their first
PREFIX_STEPS steps here (labels and the recorded logits inside the prefix), so the CPU suite
stays within minutes; gen_golden.py asserted the whole run bit-identical when it wrote them."""
import numpy as np
import pytest

from conftest import golden_case, golden_meta, hparams_of, is_continuous, state_dict_of, wave_equal

ALL = golden_meta(None)
FULL = [k for k, v in ALL.items() if v['seq_len'] * v['num_folds'] > 100000]
FAST = [k for k, v in ALL.items() if v['seq_len'] * v['num_folds'] <= 25000]
SLOW = [k for k in ALL if k not in FAST and k not in FULL]
PREFIX_STEPS = 800


def run_oracle(name, max_steps=None):
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.synth import synth_mel
    meta, gold = golden_case(name)
    hp = hparams_of(meta)
    sd = state_dict_of(meta)
    mel = synth_mel(meta['n_frames'], meta['mel_seed'])
    o = oracle_infer_waveform(sd, hp, meta['model_type'], mel, batched=meta['batched'],
                              target=meta['target'], overlap=meta['overlap'],
                              seed=meta['noise_seed'], stream=meta['stream'], max_steps=max_steps,
                              record_logits=set(int(s) for s in gold['logits_steps']))
    return meta, gold, o


def check(name):
    meta, gold, o = run_oracle(name)
    assert (o['B'], o['S']) == (meta['num_folds'], meta['seq_len'])
    if not is_continuous(meta):  # RAW / geneing BITS: categorical labels
        assert np.array_equal(o['labels'], gold['labels'])
    else:
        assert np.array_equal(o['samples'], gold['samples'])
    for i, s in enumerate(gold['logits_steps']):
        assert np.array_equal(o['logits'][int(s)], gold['logits'][i])
    assert wave_equal(o['wav'], gold)


@pytest.mark.parametrize('name', FULL)
def test_oracle_matches_reference_golden_prefix(name):
    meta, gold, o = run_oracle(name, max_steps=PREFIX_STEPS)
    assert np.array_equal(o['labels'], gold['labels'][:, :PREFIX_STEPS])
    n = 0
    for i, s in enumerate(gold['logits_steps']):
        if int(s) < PREFIX_STEPS:
            assert np.array_equal(o['logits'][int(s)], gold['logits'][i])
            n += 1
    assert n >= 2


@pytest.mark.parametrize('name', FAST)
def test_oracle_matches_reference_golden(name):
    check(name)


@pytest.mark.slow
@pytest.mark.parametrize('name', SLOW)
def test_oracle_matches_reference_golden_long(name):
    check(name)
