"""The wide-row persistent launch (kernels_persist_wide.hip: 16 rows per XCD group, fp32 MFMA
products, distributed GRU1, five hops per step) against the reference's golden outputs and the
oracle. ``WRNN_PERSIST_WIDE=1`` makes every launch of a call wide (1..16 rows per group);
the default plan picks wide, register-resident or time-sliced wide launches by cost (C4: 11
time-sliced wide launches of 16 rows per group).

Reference step: vocoder/models/fatchord_version.py:192-236; bar: bit-exact 9-bit labels.
"""
import os

import numpy as np
import pytest

from conftest import golden_case, wave_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def wide_only():
    old = os.environ.get('WRNN_PERSIST_WIDE')
    os.environ['WRNN_PERSIST_WIDE'] = '1'
    yield
    if old is None:
        del os.environ['WRNN_PERSIST_WIDE']
    else:
        os.environ['WRNN_PERSIST_WIDE'] = old


def _stage_names(m):
    return [s[0] for s in m.stage_info()]


@pytest.mark.parametrize('name', ['fatchord_raw9_tiny', 'fatchord_raw9_sharp_tiny',
                                  'fatchord_raw9_config1', 'fatchord_raw9_c2_peaked',
                                  'fatchord_raw10_defaults', 'fatchord_raw10_unbatched_tiny'])
def test_wide_golden_bit_exact(name, wide_only):
    """(10-bit: the 1024-class instances, a second fc3 tile per slot streamed from L2)"""
    meta, gold = golden_case(name)
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    m.enable_stage_timing(True)
    mel = synth_mel(meta['n_frames'], meta['mel_seed']) / sp.max_abs_value
    wav = m.generate(mel[None], meta['batched'], meta['target'], meta['overlap'], hp.mu_law,
                     sp.preemphasize, progress_callback=lambda *a: None)
    assert _stage_names(m) == ['persist_wide']
    assert np.array_equal(m.last_labels, gold['labels'])
    assert wave_equal(wav, gold)


@pytest.mark.parametrize('n_utts', [3, 13, 26])
def test_wide_row_counts_match_oracle(n_utts, wide_only):
    """5 fold rows per utterance -> 15 / 65 / 130 rows: 2, 9 and 16 + 1 rows per group (the
    last over two wide launches), every row against the oracle."""
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, hp, sd = make_model(meta)
    mels = [synth_mel(meta['n_frames'], 400 + u) / sp.max_abs_value for u in range(n_utts)]
    dev = [torch.from_numpy(x.astype(np.float32)).cuda() for x in mels]
    m.set_engine('persist')
    m.set_seed(meta['noise_seed'])
    m.enable_stage_timing(True)
    lab, roff, S = m.generate_batch_device(dev, True, meta['target'], meta['overlap'])
    assert _stage_names(m) == ['persist_wide']
    lab = lab.cpu().numpy()
    for u in sorted({0, n_utts // 2, n_utts - 1}):
        ref = oracle_infer_waveform(sd, hp, meta['model_type'], mels[u] * sp.max_abs_value,
                                    target=meta['target'], overlap=meta['overlap'],
                                    seed=meta['noise_seed'], stream=u)
        got = lab[roff[u]:roff[u + 1]]
        d = np.argwhere(got != ref['labels'])
        assert len(d) == 0, f'utt {u}: first divergence {d[np.argmin(d[:, 1])] if len(d) else None}'


def test_default_plan_uses_wide_launch_for_c4_rows():
    """144 rows (C4 per GPU) -> wide launches (time-sliced since round 5)."""
    import torch
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, hp, sd = make_model(meta)
    mels = [torch.from_numpy((synth_mel(1000, u) / sp.max_abs_value).astype(np.float32)).cuda()
            for u in range(8)]
    m.enable_stage_timing(True)
    out, roff, S = m.generate_batch_device(mels, True, 11000, 550)
    assert roff[-1] == 144
    names = _stage_names(m)
    assert 'persist_wide' in names, names


def test_wide_every_rows_per_group_matches_register_resident(monkeypatch):
    """Every group fill of the wide launch, 1..16 rows per group, with padding rows in some
    groups (8 R - R % 3 unbatched 1-row utterances): the wide kernel's labels equal the
    register-resident kernel's (itself pinned to the oracle) row for row. The row counts the
    round-3 18-row instance deadlocked at do not exist in the shipped kernel (<= 16); this covers
    the shipped instance's."""
    import torch
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw9_tiny')
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    m.enable_stage_timing(True)
    for R in range(1, 17):
        n = 8 * R - R % 3
        dev = [torch.from_numpy((synth_mel(6, 700 + u) / sp.max_abs_value).astype(np.float32)).cuda()
               for u in range(n)]
        out = {}
        for wide in ('1', '0'):
            monkeypatch.setenv('WRNN_PERSIST_WIDE', wide)
            m.set_seed(meta['noise_seed'])
            lab, roff, S = m.generate_batch_device(dev, False, 0, 0)
            names = _stage_names(m)
            assert ('persist_wide' in names) == (wide == '1'), (R, wide, names)
            out[wide] = lab.cpu().numpy()
        d = np.argwhere(out['1'] != out['0'])
        assert len(d) == 0, f'R={R} ({n} rows): first divergence {d[np.argmin(d[:, 1])]}'


@pytest.mark.parametrize('case', ['fatchord_raw9_sharp_tiny', 'fatchord_raw10_unbatched_tiny'])
def test_wide_p1_ring_equals_stream(case, wide_only, monkeypatch):
    """The wide kernel forms P1 in its one-slot LDS ring from the per-frame tables (p1_make) or,
    with WRNN_P1_RING=0, copies it from k_p1_expand's [S][B][4H] stream: identical labels
    (9-bit and the 1024-class instances)."""
    import torch
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case(case)
    m, hp, sd = make_model(meta)
    m.set_engine('persist')
    m.enable_stage_timing(True)
    dev = [torch.from_numpy((synth_mel(meta['n_frames'], 300 + u) / sp.max_abs_value).astype(np.float32)).cuda()
           for u in range(4)]
    out = []
    for ring in ('1', '0'):
        monkeypatch.setenv('WRNN_P1_RING', ring)
        m.set_seed(meta['noise_seed'])
        res, roff, S = m.generate_batch_device(dev, meta['batched'], meta['target'], meta['overlap'])
        assert _stage_names(m) == ['persist_wide']
        out.append(res.cpu().numpy())
    d = np.argwhere(out[0] != out[1])
    assert len(d) == 0, f'first divergence {d[np.argmin(d[:, 1])].tolist()}'


def test_wide_10bit_time_sliced_batch_matches_oracle():
    """fatchord 10-bit (1024 classes) at target 3000 / overlap 1500, 8 utterances of 17 fold rows
    (136 rows, 17 per group): 17 time-sliced wide launches of 16 rows per group x 375 steps on the
    1024-class instances (each row in 16 of them, its state carried across); utterances 0 and 7
    against the oracle, every label of all 6,000 steps."""
    import torch
    from oracle.wavernn_oracle import oracle_infer_waveform
    from test_gpu_parity import make_model
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    meta, _ = golden_case('fatchord_raw10_defaults')
    m, hp, sd = make_model(meta)
    T = next(t for t in range(2, 2000) if m.fold_shape(t, True, 3000, 1500)[0] == 17)
    mels = [synth_mel(T, 700 + u) / sp.max_abs_value for u in range(8)]
    dev = [torch.from_numpy(x.astype(np.float32)).cuda() for x in mels]
    m.set_engine('persist')
    m.set_seed(meta['noise_seed'])
    m.enable_stage_timing(True)
    lab, roff, S = m.generate_batch_device(dev, True, 3000, 1500)
    plan = m.plan_info()
    assert roff[-1] == 136 and S == 6000 and plan == [(0, 16, True)] * 17, (roff, S, plan)
    lab = lab.cpu().numpy()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    for u in (0, 7):
        ref = oracle_infer_waveform(sd, hp, meta['model_type'], mels[u] * sp.max_abs_value,
                                    target=3000, overlap=1500, seed=meta['noise_seed'], stream=u)
        got = lab[roff[u]:roff[u + 1]]
        d = np.argwhere(got != ref['labels'])
        assert len(d) == 0, f'utt {u}: first divergence {d[np.argmin(d[:, 1])].tolist() if len(d) else None}'
