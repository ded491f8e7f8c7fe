"""Fold-range calls (wrnn_set_fold_ranges): the single-utterance split of SURVEY §8e.

A rank of a fold-split job (wavernn_amd.distributed, split='folds') runs only fold rows
lo .. hi - 1 of an utterance. Every such row must be the row the whole-utterance call produces:
same conditioning positions (fold_with_overlap, fatchord_version.py:290-340), same noise words
(Philox keyed by the global fold index). Checked here against whole calls at C2's full size
(18 x 12,100) for the cuts a 2-, 3- and 4-GPU split makes and for edge ranges, against the
oracle for a cut's rows, on the MOL path, on a multi-utterance call whose ranged rows run the
time-sliced wide launches, and for the argument errors. The register-resident kernels give
every row the same arithmetic at any rows-per-group count, so at C2 the
ranged rows equal the whole call's bit for bit (labels and MOL samples); rows that move
between the wide and the register-resident family compare as labels (both bit-exact against
the oracle on these seeds).
"""
import numpy as np
import pytest

from test_gpu_fullsize import FRAMES, NOISE_SEED, OVERLAP, TARGET, device_mels, first_divergence, make, oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def c2():
    m, hp, sd = make()
    m.set_seed(NOISE_SEED)
    mel = device_mels([0])
    full, roff, S = m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[0])
    assert m.last_engine() == 'persist' and roff == [0, 18] and S == 12100
    return m, hp, sd, mel, full.cpu().numpy()


@pytest.mark.parametrize('ranges', [
    [(0, 9), (9, 18)],               # 2 GPUs: 9 rows each (rotated groups of 2 and 1 rows)
    [(0, 6), (6, 12), (12, 18)],     # 3 GPUs: one row per XCD group
    [(0, 4), (4, 9), (9, 13), (13, 18)],
    [(17, 18), (0, 1), (3, 16)],     # the zero-padded tail fold alone, fold 0 alone, a middle run
])
def test_ranges_equal_whole_call(c2, ranges):
    m, _, _, mel, full = c2
    for lo, hi in ranges:
        out, roff, S = m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[0],
                                               fold_ranges=[(lo, hi)])
        assert m.last_engine() == 'persist'
        assert roff == [0, hi - lo] and S == 12100
        got = out.cpu().numpy()
        assert np.array_equal(got, full[lo:hi]), \
            f'[{lo}, {hi}): first divergence (row, step) {first_divergence(got, full[lo:hi])}'


def test_split_rows_match_oracle(c2):
    """The second half of a 2-GPU split against the oracle (the reference restated)."""
    m, hp, sd, mel, _ = c2
    out, _, _ = m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[0], fold_ranges=[(9, 18)])
    ref = oracle(sd, hp, 'fatchord-wavernn', 0, stream=0)['labels'][9:18]
    got = out.cpu().numpy()
    assert np.array_equal(got, ref), f'first divergence (row, step) {first_divergence(got, ref)}'


def test_three_gpu_split_plan_is_one_row_per_group(c2):
    m, _, _, mel, _ = c2
    m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[0], fold_ranges=[(6, 12)])
    plan = m.plan_info()
    assert plan and all(nr == 1 and not wide for _, nr, wide in plan), plan


def test_mol_ranges_equal_whole_call():
    m, _, _ = make(mode='MOL')
    m.set_seed(NOISE_SEED)
    mel = device_mels([3])
    full, _, _ = m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[2])
    full = full.cpu().numpy()
    for lo, hi in [(0, 9), (9, 18)]:
        out, _, _ = m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[2], fold_ranges=[(lo, hi)])
        assert np.array_equal(out.cpu().numpy(), full[lo:hi])


def test_multi_utterance_ranges_on_the_wide_kernel():
    """8 utterances (C4's per-GPU shape) cut as a 2-GPU fold split of 16 utterances would cut
    them: 72 of the 144 rows, every utterance split at fold 9 -- the time-sliced wide launches."""
    m, _, _ = make()
    m.set_seed(NOISE_SEED)
    mels = device_mels(range(8))
    full, roff, _ = m.generate_batch_device(mels, True, TARGET, OVERLAP, streams=list(range(8)))
    full = full.cpu().numpy()
    ranges = [(0, 9) if u % 2 == 0 else (9, 18) for u in range(8)]
    out, roff2, _ = m.generate_batch_device(mels, True, TARGET, OVERLAP, streams=list(range(8)),
                                            fold_ranges=ranges)
    assert roff2 == [9 * u for u in range(9)]
    assert any(wide for _, _, wide in m.plan_info())
    got = out.cpu().numpy()
    for u, (lo, hi) in enumerate(ranges):
        want = full[roff[u] + lo:roff[u] + hi]
        assert np.array_equal(got[roff2[u]:roff2[u + 1]], want), \
            f'utt {u}: first divergence {first_divergence(got[roff2[u]:roff2[u + 1]], want)}'


def test_range_errors_and_one_shot(c2):
    m, _, _, mel, full = c2
    for bad in [(0, 19), (5, 5), (-1, 3)]:
        with pytest.raises(ValueError):
            m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[0], fold_ranges=[bad])
    with pytest.raises(ValueError):
        m.generate_batch_device(mel, True, TARGET, OVERLAP, fold_ranges=[(0, 9), (9, 18)])
    # the single-utterance host call refuses an armed range and disarms it
    import ctypes
    lo, hi = (ctypes.c_int * 1)(0), (ctypes.c_int * 1)(9)
    assert m._lib.wrnn_set_fold_ranges(m._h, lo, hi, 1) == 0
    from wavernn_amd.synth import synth_mel
    with pytest.raises(ValueError):
        m.generate_rows(synth_mel(FRAMES, 0) / 4.0, True, TARGET, OVERLAP)
    # ... and a failed or refused call leaves nothing armed: the next call is a whole one
    out, roff, _ = m.generate_batch_device(mel, True, TARGET, OVERLAP, streams=[0])
    assert roff == [0, 18] and np.array_equal(out.cpu().numpy(), full)
