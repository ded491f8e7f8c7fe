"""The runtimeracer wide-row launch (kernels_persist_wide_rr.hip: 16 rows per XCD group, the
group split into two halves of 16 slots owning alternate layers, fp32 MFMA products, nine hops
per step) against the reference's golden outputs, the oracle and the register-resident
runtimeracer kernel. ``WRNN_PERSIST_WIDE=1`` makes every launch of a call wide.

Reference step: vocoder/models/runtimeracer_version.py:244-270; bar: bit-exact labels (9 / 10 bit).
"""
import numpy as np
import pytest

from conftest import golden_case, wave_equal

pytestmark = pytest.mark.gpu


def _names(m):
    return [s[0] for s in m.stage_info()]


@pytest.mark.parametrize('name', ['runtimeracer_raw9_tiny', 'runtimeracer_raw10_defaults'])
def test_wide_rr_golden_bit_exact(name, monkeypatch):
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    monkeypatch.setenv('WRNN_PERSIST_WIDE', '1')
    meta, gold = golden_case(name)
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    m.enable_stage_timing(True)
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    wav = m.generate(mel[None], meta['batched'], meta['target'], meta['overlap'], hp.mu_law,
                     sp.preemphasize, progress_callback=lambda *a: None)
    assert _names(m) == ['persist_wide']
    lab = m.last_labels
    d = np.argwhere(lab != gold['labels'])
    assert len(d) == 0, f'first divergence {d[np.argmin(d[:, 1])].tolist()}'
    assert wave_equal(wav, gold)


def test_wide_rr_every_rows_per_group_matches_register_resident(monkeypatch):
    """1..16 rows per group (8 R - R % 3 unbatched 1-row utterances, so some groups carry padding
    rows): wide labels equal the register-resident runtimeracer kernel's row for row."""
    import torch
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('runtimeracer_raw9_tiny')
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    m.enable_stage_timing(True)
    for R in (1, 2, 3, 5, 8, 11, 13, 16):
        n = 8 * R - R % 3
        dev = [torch.from_numpy((synth_mel(6, 900 + u) / sp.max_abs_value).astype(np.float32)).cuda()
               for u in range(n)]
        out = {}
        for wide in ('1', '0'):
            monkeypatch.setenv('WRNN_PERSIST_WIDE', wide)
            m.set_seed(meta['noise_seed'])
            lab, roff, S = m.generate_batch_device(dev, False, 0, 0)
            assert ('persist_wide' in _names(m)) == (wide == '1'), (R, wide, _names(m))
            out[wide] = lab.cpu().numpy()
        d = np.argwhere(out['1'] != out['0'])
        assert len(d) == 0, f'R={R} ({n} rows): first divergence {d[np.argmin(d[:, 1])]}'


def test_wide_rr_c4_shape_10bit_defaults_matches_oracle():
    """The fork's default topology and config at the C4 per-GPU shape: 8 x 1000-frame mels,
    runtimeracer RAW 10-bit, target 6000 / overlap 1000 (8 x 29 = 232 fold rows) in one call
    with the default launch plan; utterances 0 and 7 against the oracle, every label."""
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from test_gpu_fullsize import make
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp, sd = make(model_type='runtimeracer-wavernn', bits=10, weight_seed=8)
    m.set_seed(4321)
    m.enable_stage_timing(True)
    mels = [synth_mel(1000, 50 + u) for u in range(8)]
    dev = [torch.from_numpy((x / sp.max_abs_value).astype(np.float32)).cuda() for x in mels]
    out, roff, S = m.generate_batch_device(dev, True, hp.gen_target, hp.gen_overlap)
    assert m.last_engine() == 'persist' and roff[-1] == 232 and S == 8000
    print('launch plan stages', m.stage_info())
    assert 'persist_wide' in _names(m)
    lab = out.cpu().numpy()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    for u in (0, 7):
        ref = oracle_infer_waveform(sd, hp, 'runtimeracer-wavernn', mels[u], target=hp.gen_target,
                                    overlap=hp.gen_overlap, seed=4321, stream=u)
        got = lab[roff[u]:roff[u + 1]]
        d = np.argwhere(got != ref['labels'])
        assert len(d) == 0, f'utt {u}: first divergence {d[np.argmin(d[:, 1])].tolist()}'
