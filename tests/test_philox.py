"""Philox4x32-10 noise contract (oracle/philox.py) -- Random123 known-answer vectors and the
properties the sampler relies on. CPU only."""
import numpy as np

from oracle import philox


KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


def test_random123_known_answers():
    for c, k, exp in KAT:
        got = tuple(int(x) for x in philox.philox4x32_10(*c, *k))
        assert got == exp


def test_raw_noise_is_exp1_and_positive():
    q = philox.raw_exp_noise(7, 3, np.arange(200), np.arange(4), 512).astype(np.float64)
    assert q.shape == (200, 4, 512)
    assert (q > 0).all() and np.isfinite(q).all()
    assert abs(q.mean() - 1.0) < 0.01 and abs(q.var() - 1.0) < 0.03


def test_noise_streams_are_distinct_and_reproducible():
    a = philox.raw_exp_noise(1, 0, [5], [0, 1], 64)
    assert np.array_equal(a, philox.raw_exp_noise(1, 0, [5], [0, 1], 64))
    assert not np.array_equal(a[0, 0], a[0, 1])                       # rows
    assert not np.array_equal(a, philox.raw_exp_noise(1, 1, [5], [0, 1], 64))  # stream
    assert not np.array_equal(a, philox.raw_exp_noise(2, 0, [5], [0, 1], 64))  # seed


def test_mol_uniforms_range():
    u1, u2 = philox.mol_uniforms(0, 0, np.arange(100), np.arange(3))
    assert u1.shape == (100, 3, 10) and u2.shape == (100, 3)
    for u in (u1, u2):
        assert (u >= np.float32(1e-5)).all() and (u <= np.float32(1 - 1e-5)).all()


def test_beta_samples_follow_beta_distribution():
    """BETA contract (geneing 'RAW', vocoder/distribution.py:7-20): 2 Beta(a, b) - 1 with the
    right first two moments, for shapes above and below 1 (the a < 1 boost path)."""
    rows = np.arange(20000)
    for a, b in ((2.0, 5.0), (0.5, 0.7), (30.0, 3.0), (1.0, 1.0)):
        x = philox.beta_sample(11, 2, 7, rows, np.full(rows.shape, a, np.float32),
                               np.full(rows.shape, b, np.float32)).astype(np.float64)
        assert ((x >= -1) & (x <= 1)).all()
        s = (x + 1) / 2
        mean, var = a / (a + b), a * b / ((a + b) ** 2 * (a + b + 1))
        assert abs(s.mean() - mean) < 5 * np.sqrt(var / len(rows)) + 1e-4, (a, b)
        assert abs(s.var() - var) < 0.05 * var, (a, b)


def test_beta_streams_are_distinct_and_reproducible():
    al = np.full(4, 2.0, np.float32)
    x = philox.beta_sample(1, 0, 5, np.arange(4), al, al)
    assert np.array_equal(x, philox.beta_sample(1, 0, 5, np.arange(4), al, al))
    assert len(set(x.tolist())) == 4
    assert not np.array_equal(x, philox.beta_sample(1, 1, 5, np.arange(4), al, al))
    assert not np.array_equal(x, philox.beta_sample(1, 0, 6, np.arange(4), al, al))
