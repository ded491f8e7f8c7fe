"""Pins the oracle: the torch-CPU restatement reproduces, bit for bit, the outputs the REAL
reference generate() produced (tests/golden/*.npz, written by tests/golden/gen_golden.py in the
survey container with the reference imported from /root/reference). CPU only."""
import numpy as np
import pytest

from conftest import golden_case, golden_meta, hparams_of, is_continuous

FAST = [k for k, v in golden_meta().items() if v['seq_len'] * v['num_folds'] <= 25000]
SLOW = [k for k in golden_meta() if k not in FAST]


def run_oracle(name):
    from oracle.wavernn_oracle import oracle_infer_waveform
    from wavernn_amd.synth import synth_state_dict, synth_mel
    meta, gold = golden_case(name)
    hp = hparams_of(meta)
    sd = synth_state_dict(hp, meta['model_type'], seed=meta['weight_seed'],
                          logit_scale=meta['logit_scale'])
    mel = synth_mel(meta['n_frames'], meta['mel_seed'])
    o = oracle_infer_waveform(sd, hp, meta['model_type'], mel, batched=meta['batched'],
                              target=meta['target'], overlap=meta['overlap'],
                              seed=meta['noise_seed'], stream=meta['stream'],
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
    assert np.array_equal(o['wav'], gold['wav'])


@pytest.mark.parametrize('name', FAST)
def test_oracle_matches_reference_golden(name):
    check(name)


@pytest.mark.slow
@pytest.mark.parametrize('name', SLOW)
def test_oracle_matches_reference_golden_long(name):
    check(name)
