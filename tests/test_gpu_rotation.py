"""Row rotation and time-sliced wide launches (§3.0f) on the GPU: a call whose rows leave the
XCD groups uneven (R % 8 != 0) runs as K launches over rotating row sets, groups of q rows on
their own q-row body. The rotation only moves WHERE and WHEN a row's steps run: every row's
arithmetic is the same, so the labels / samples must equal the single-launch plan's
(WRNN_PERSIST_ROT=0) bit for bit -- RAW and MOL, several row counts, with logit capture (the
DBG instances) and with the reference's progress callback. Full-size parity against the oracle
with the rotation on is tests/test_gpu_fullsize.py (C2 is rotated by default).
Reference: vocoder/models/fatchord_version.py:192-236 (the step), :234-236 (progress)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TARGET, OVERLAP = 4000, 400  # 4,800 steps (shorter calls do not pay for the extra launches)


def _model(mode='RAW', bits=9, model_type='fatchord-wavernn'):
    from wavernn_amd.base import hparams_for
    from wavernn_amd.hparams import sp
    from wavernn_amd.model import WaveRNN
    from wavernn_amd.synth import synth_state_dict
    hp = hparams_for(model_type).copy(bits=bits, mode=mode)
    m = WaveRNN(hp.rnn_dims, hp.fc_dims, hp.bits, hp.pad, hp.upsample_factors, sp.num_mels, hp.compute_dims,
                hp.res_out_dims, hp.res_blocks, sp.hop_size, sp.sample_rate, mode=mode,
                model_type=model_type, device=0)
    m.load_state_dict(synth_state_dict(hp, model_type, seed=11))
    m.set_engine('persist')
    return m, hp


def _frames_for(m, rows):
    for T in range(2, 2000):
        if m.fold_shape(T, True, TARGET, OVERLAP)[0] == rows:
            return T
    raise AssertionError(rows)


def _call(m, mel, monkeypatch, rot, debug_steps=None, cb=None):
    import torch
    from wavernn_amd.hparams import sp
    monkeypatch.setenv('WRNN_PERSIST_ROT', '1' if rot else '0')
    m.set_seed(77)
    m.set_debug_steps(debug_steps)
    try:
        if cb is None:
            dev = torch.from_numpy((mel / sp.max_abs_value).astype(np.float32)).cuda()
            out, roff, S = m.generate_batch_device([dev], True, TARGET, OVERLAP)
            res = out.cpu().numpy()
        else:
            m.generate((mel / sp.max_abs_value)[None], True, TARGET, OVERLAP, True, True, progress_callback=cb)
            res = m.last_labels if m.last_labels is not None else m.last_samples
        logs = {s: m.debug_logits(s, range(res.shape[0])) for s in (debug_steps or [])}
        return res, m.rot_info(), logs
    finally:
        m.set_debug_steps(None)


@pytest.mark.parametrize('rows', [9, 10, 17, 18, 20])
def test_rotated_labels_equal_single_launch(rows, monkeypatch):
    from wavernn_amd.synth import synth_mel
    m, hp = _model()
    mel = synth_mel(_frames_for(m, rows), 500 + rows)
    a, ra, _ = _call(m, mel, monkeypatch, rot=True)
    b, rb, _ = _call(m, mel, monkeypatch, rot=False)
    assert a.shape[0] == rows and ra[0] > 1 and rb[0] == 0, (a.shape, ra, rb)
    d = np.argwhere(a != b)
    assert len(d) == 0, f'{rows} rows: first difference {d[np.argmin(d[:, 1])].tolist()}'


@pytest.mark.parametrize('model_type,rows', [('fatchord-wavernn', 18), ('geneing-wavernn', 18),
                                             ('geneing-wavernn', 20), ('runtimeracer-wavernn', 18),
                                             ('runtimeracer-wavernn', 17)])
def test_rotated_mol_samples_equal_single_launch(model_type, rows, monkeypatch):
    """MOL rotated (k_persist / k_persist_gen / k_persist_rr <..., MOL, ROT>: the 11 noise draws and the sample
    column at each row's own step): samples, and the logits around the launch boundaries, equal
    the single launch's bit for bit."""
    from wavernn_amd.synth import synth_mel
    m, hp = _model('MOL', model_type=model_type)
    mel = synth_mel(_frames_for(m, rows), 77)
    _, (K, nh, nl), _ = _call(m, mel, monkeypatch, rot=True)
    steps = [0, nh - 1, nh, nl, nh + nl - 1, nh + nl, 2 * nl, 4799]
    a, ra, la = _call(m, mel, monkeypatch, rot=True, debug_steps=steps)
    b, rb, lb = _call(m, mel, monkeypatch, rot=False, debug_steps=steps)
    assert a.shape[0] == rows and ra[0] > 1 and rb[0] == 0, (a.shape, ra, rb)
    assert np.array_equal(a, b)
    for s in steps:
        assert np.isfinite(la[s]).all(), s
        assert np.array_equal(la[s], lb[s]), s


def test_rotated_logit_capture_equals_single_launch(monkeypatch):
    """The DBG instances record each row's logits at its own step (the offset step)."""
    from wavernn_amd.synth import synth_mel
    m, hp = _model()
    mel = synth_mel(_frames_for(m, 18), 3)
    # around the launch boundaries (18 rows, 4,800 steps: n_hi steps at 3 rows, n_lo at 2; a
    # row's offsets are 0, n_hi or n_lo, n_hi + n_lo or 2 n_lo)
    _, (K, nh, nl), _ = _call(m, mel, monkeypatch, rot=True)
    steps = [0, nh - 1, nh, nl, nh + nl - 1, nh + nl, 2 * nl, 4799]
    a, ra, la = _call(m, mel, monkeypatch, rot=True, debug_steps=steps)
    b, rb, lb = _call(m, mel, monkeypatch, rot=False, debug_steps=steps)
    assert ra[0] > 1 and np.array_equal(a, b)
    for s in steps:
        assert np.isfinite(la[s]).all(), s
        assert np.array_equal(la[s], lb[s]), s


def test_rotated_call_reports_progress_at_the_reference_cadence(monkeypatch):
    from wavernn_amd.synth import synth_mel
    m, hp = _model()
    mel = synth_mel(_frames_for(m, 18), 5)
    seen = []
    a, ra, _ = _call(m, mel, monkeypatch, rot=True, cb=lambda i, n, b, r: seen.append((i, n, b)))
    S = a.shape[1]
    assert ra[0] > 1
    assert [s[0] for s in seen] == list(range(0, S, 100))
    assert all(n == S and b == 18 for _, n, b in seen)
    b_, rb, _ = _call(m, mel, monkeypatch, rot=False)
    assert np.array_equal(a, b_)


@pytest.mark.parametrize('model_type,bits', [('fatchord-wavernn', 9), ('fatchord-wavernn', 10),
                                             ('runtimeracer-wavernn', 10)])
def test_time_sliced_wide_equals_wide_plus_tail(model_type, bits, monkeypatch):
    """8 utterances x 18 rows (the C4 shape at 4,800 steps): the time-sliced wide launches (every
    row through 16-row-per-group wide launches at its own offsets, state across launches) give
    the labels of the wide 128-row launch + register-resident 16-row launch plan
    (WRNN_PERSIST_SLICE=0) bit for bit, and so do the wide rows' logits recorded around the slice
    boundaries (600 steps per launch at 4,800 steps: 8 of 9 launches per row). fatchord 10 bits:
    the 1024-class instances; runtimeracer: the two-half kernel (kernels_persist_wide_rr.hip),
    its four GRUs' state (and gh4) across launches."""
    import torch
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp = _model(bits=bits, model_type=model_type)
    T = _frames_for(m, 18)
    devs = [torch.from_numpy((synth_mel(T, 40 + u) / sp.max_abs_value).astype(np.float32)).cuda() for u in range(8)]
    steps = [0, 599, 600, 601, 1199, 1200, 2400, 4799]
    res = {}
    for sl in ('1', '0'):
        monkeypatch.setenv('WRNN_PERSIST_SLICE', sl)
        m.set_seed(9)
        m.set_debug_steps(steps)
        try:
            out, roff, S = m.generate_batch_device(devs, True, TARGET, OVERLAP)
            lab = out.cpu().numpy()
            logs = {s: m.debug_logits(s, range(lab.shape[0])) for s in steps}
        finally:
            m.set_debug_steps(None)
        res[sl] = (lab, logs, m.plan_info())
    (a, la, pa), (b, lb, pb) = res['1'], res['0']
    assert len(pa) > 2 and all(w for _, _, w in pa) and any(not w for _, _, w in pb), (pa, pb)
    d = np.argwhere(a != b)
    assert len(d) == 0, f'first difference (row, step) {d[np.argmin(d[:, 1])].tolist()}'
    # (logits: the rows both plans run on the wide kernel -- the other plan's 16 register-resident
    # rows, wherever its launch order puts them, run a different fp32 summation order)
    wide = np.concatenate([np.arange(rb, rb + 8 * nr) for rb, nr, w in pb if w])
    assert len(wide) == 128
    bad = []
    for s in steps:
        dr = [int(r) for r in wide if not np.array_equal(la[s][r], lb[s][r])]
        if dr:
            dd = np.abs(la[s][dr] - lb[s][dr])
            bad.append((s, len(dr), dr[:20], float(dd.max()), int((dd > 0).sum())))
    assert not bad, (bad, pa, pb)


def test_time_sliced_call_reports_progress_in_order(monkeypatch):
    """A time-sliced call (8 x 18 rows) with the reference's progress callback: i = 0, 100, ...
    < S exactly once each, in order, with (S, b_size) of the call, and the labels of the call
    without a callback (the kernels only publish a progress word)."""
    import torch
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp = _model()
    T = _frames_for(m, 18)
    devs = [torch.from_numpy((synth_mel(T, 60 + u) / sp.max_abs_value).astype(np.float32)).cuda() for u in range(8)]
    seen = []
    m.set_seed(5)
    a, _, S = m.generate_batch_device(devs, True, TARGET, OVERLAP,
                                      progress_callback=lambda i, n, b, r: seen.append((i, n, b)))
    assert len(m.plan_info()) > 2 and all(w for _, _, w in m.plan_info())
    m.set_seed(5)
    b, _, _ = m.generate_batch_device(devs, True, TARGET, OVERLAP)
    assert [s[0] for s in seen] == list(range(0, S, 100))
    assert all(n == S and bb == 144 for _, n, bb in seen)
    assert torch.equal(a, b)


def test_time_sliced_ragged_utterances_equal_unsliced(monkeypatch):
    """Eight utterances of different lengths (17-20 fold rows each, 144 in all: ragged tail folds,
    rows of one utterance in several groups) through the time-sliced wide launches: labels equal
    the unsliced plan's bit for bit, utterance by utterance."""
    import torch
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp = _model()
    counts = [17, 19, 18, 18, 20, 16, 18, 18]
    devs = [torch.from_numpy((synth_mel(_frames_for(m, c), 80 + u) / sp.max_abs_value).astype(np.float32)).cuda()
            for u, c in enumerate(counts)]
    res = {}
    for sl in ('1', '0'):
        monkeypatch.setenv('WRNN_PERSIST_SLICE', sl)
        m.set_seed(21)
        out, roff, S = m.generate_batch_device(devs, True, TARGET, OVERLAP)
        res[sl] = (out.cpu().numpy(), list(roff), m.plan_info())
    (a, ra, pa), (b, rb, pb) = res['1'], res['0']
    assert ra == rb and ra[-1] == 144 and len(pa) > 2 and all(w for _, _, w in pa), (ra, pa)
    for u in range(len(counts)):
        d = np.argwhere(a[ra[u]:ra[u + 1]] != b[rb[u]:rb[u + 1]])
        assert len(d) == 0, f'utterance {u}: first difference {d[np.argmin(d[:, 1])].tolist()}'


def test_rotated_ragged_utterances_equal_single_launch(monkeypatch):
    """Two utterances of 9 and 8 fold rows (17 rows: one group of 3, seven of 2) rotated: labels
    equal the single launch's."""
    import torch
    from wavernn_amd.hparams import sp
    from wavernn_amd.synth import synth_mel
    m, hp = _model()
    devs = [torch.from_numpy((synth_mel(_frames_for(m, c), 90 + u) / sp.max_abs_value).astype(np.float32)).cuda()
            for u, c in enumerate((9, 8))]
    res = {}
    for rot in ('1', '0'):
        monkeypatch.setenv('WRNN_PERSIST_ROT', rot)
        m.set_seed(23)
        out, roff, S = m.generate_batch_device(devs, True, TARGET, OVERLAP)
        res[rot] = (out.cpu().numpy(), m.rot_info())
    assert res['1'][1][0] > 1 and res['0'][1][0] == 0, (res['1'][1], res['0'][1])
    d = np.argwhere(res['1'][0] != res['0'][0])
    assert len(d) == 0, f'first difference {d[np.argmin(d[:, 1])].tolist()}'


@pytest.mark.parametrize('model_type,mode,bits,rows', [
    ('runtimeracer-wavernn', 'RAW', 9, 18), ('runtimeracer-wavernn', 'RAW', 10, 20),
    ('runtimeracer-wavernn', 'RAW', 9, 17),
    ('geneing-wavernn', 'BITS', 10, 18), ('geneing-wavernn', 'BITS', 9, 20), ('geneing-wavernn', 'BITS', 10, 17)])
def test_rotated_runtimeracer_geneing_labels_equal_single_launch(model_type, mode, bits, rows, monkeypatch):
    """The runtimeracer / geneing register-resident kernels rotated (k_persist_rr / k_persist_gen
    <..., ROT>: rows at their own step offsets, the GRUs' chunk state across launches, P1 and the
    noise streams read at each row's own step): labels, and the logits recorded around the launch
    boundaries, equal the single launch's bit for bit."""
    from wavernn_amd.synth import synth_mel
    m, hp = _model(mode=mode, bits=bits, model_type=model_type)
    mel = synth_mel(_frames_for(m, rows), 600 + rows)
    _, (K, nh, nl), _ = _call(m, mel, monkeypatch, rot=True)
    steps = [0, nh - 1, nh, nl, nh + nl - 1, nh + nl, 2 * nl, 4799]
    a, ra, la = _call(m, mel, monkeypatch, rot=True, debug_steps=steps)
    b, rb, lb = _call(m, mel, monkeypatch, rot=False, debug_steps=steps)
    assert a.shape[0] == rows and ra[0] > 1 and rb[0] == 0, (a.shape, ra, rb)
    d = np.argwhere(a != b)
    assert len(d) == 0, f'{rows} rows: first difference {d[np.argmin(d[:, 1])].tolist()}'
    for s in steps:
        assert np.isfinite(la[s]).all(), s
        assert np.array_equal(la[s], lb[s]), s
