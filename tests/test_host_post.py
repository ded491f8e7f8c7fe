"""CPU only: the fast host post-processing of ``generate`` (wavernn_amd/audio.py) against the
plain restatement of the reference's (fatchord_version.py:238-255: xfade_and_unfold, then
decode_mu_law, then vocoder/audio.py:92-93 de_emphasis = scipy lfilter), bit for bit:

* the mu-law table path (fold middles looked up from the n_classes decoded label values, only
  the cross-faded overlaps decoded directly);
* ``wrnn_de_emphasis``, the library's host loop of scipy's lfilter recurrence.
"""
import numpy as np
import pytest

from wavernn_amd import _abi, audio
from wavernn_amd.model import labels_to_samples


@pytest.fixture(scope='module')
def lib():
    return _abi.load_library()


@pytest.mark.parametrize('n,B,target,overlap', [(512, 18, 11000, 550), (1024, 5, 300, 50),
                                                (512, 3, 200, 51), (512, 1, 1100, 550),
                                                (1024, 7, 600, 100), (512, 4, 40, 1)])
def test_table_and_native_post_bit_exact(lib, n, B, target, overlap):
    rng = np.random.default_rng(n + B + target)
    lab = rng.integers(0, n, (B, target + 2 * overlap)).astype(np.int16)
    smp = labels_to_samples(lab, n)
    wave_len = B * (target + overlap) + overlap - 7 * 5
    ref = audio.postprocess(smp, True, target, overlap, True, True, n, wave_len, 5)
    got = audio.postprocess(smp, True, target, overlap, True, True, n, wave_len, 5, labels=lab,
                            lib=lib)
    assert got.dtype == ref.dtype == np.float64
    assert np.array_equal(got, ref)


@pytest.mark.parametrize('size', [0, 1, 2, 17, 100003])
def test_native_de_emphasis_matches_lfilter(lib, size):
    rng = np.random.default_rng(size)
    x = rng.standard_normal(size) * 0.5
    if size > 4:
        x[1] = -0.0
        x[3] = 0.0
    ref = audio.de_emphasis(x)
    got = audio.de_emphasis_native(x, lib)
    assert np.array_equal(got, ref)
    assert np.array_equal(np.signbit(got), np.signbit(ref))


@pytest.mark.parametrize('mu_law,preemph', [(True, True), (False, True), (True, False),
                                            (False, False)])
@pytest.mark.parametrize('n,B,target,overlap,extra', [(512, 18, 11000, 550, -199),
                                                      (1024, 5, 300, 51, 0),
                                                      (512, 1, 1100, 550, 4000),
                                                      (512, 4, 40, 1, -3)])
def test_fused_label_post_bit_exact(lib, mu_law, preemph, n, B, target, overlap, extra):
    """wrnn_post_overlaps / wrnn_post_assemble (one pass over the labels) against the plain
    restatement: every mode flag, wave_len below and above the unfolded length."""
    rng = np.random.default_rng(n * B + overlap)
    lab = rng.integers(0, n, (B, target + 2 * overlap)).astype(np.int16)
    lab[0, :3] = 0
    lab[-1, -3:] = n - 1
    smp = labels_to_samples(lab, n)
    hop = 5
    wave_len = B * (target + overlap) + overlap + extra
    ref = audio.postprocess(smp, True, target, overlap, mu_law, preemph, n, wave_len, hop)
    got = audio.postprocess_labels(lab, target, overlap, mu_law, preemph, n, wave_len, hop, lib)
    assert got is not None and got.dtype == np.float64
    assert np.array_equal(got, ref)
    assert np.array_equal(np.signbit(got), np.signbit(ref))


def test_fused_label_post_edges(lib):
    lab = np.zeros((2, 30), np.int16)
    # output shorter than the final fade: not the fused path (postprocess keeps the reference's
    # own behaviour for it)
    assert audio.postprocess_labels(lab, 10, 10, True, True, 512, 19, 1, lib) is None
    lab[1, 4] = 512
    with pytest.raises(RuntimeError):
        audio.postprocess_labels(lab, 10, 10, True, True, 512, 50, 1, lib)
    lab[1, 4] = -1
    with pytest.raises(RuntimeError):
        audio.postprocess_labels(lab, 10, 10, True, True, 512, 50, 1, lib)
