"""The C-ABI library (include/wavernn_mi355x.h) loads and exports every declared symbol; host
argument checking works without a GPU. CPU only (no compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def declared_symbols():
    src = open(os.path.join(REPO, 'include', 'wavernn_mi355x.h')).read()
    return sorted(set(re.findall(r'\b(wrnn_[a-z0-9_]+)\s*\(', src)) - {'wrnn_progress_fn'})


def test_header_and_binding_agree():
    from wavernn_amd import _abi
    assert sorted(_abi.EXPORTED) == declared_symbols()


def test_library_exports_every_declared_symbol():
    from wavernn_amd import _abi
    lib = _abi.load_library()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.wrnn_version().startswith(b'wavernn-mi355x')


def test_fold_shape_matches_reference_arithmetic():
    """fold_with_overlap (fatchord_version.py:316-327) restated in the oracle vs the ABI."""
    import torch
    from oracle.wavernn_oracle import OracleWaveRNN
    from wavernn_amd import _abi
    lib = _abi.load_library()
    for T, tgt, ovl in [(1000, 11000, 550), (200, 11000, 550), (24, 1000, 100), (53, 3000, 1500),
                        (71, 6000, 1000), (1, 100, 10), (7, 50, 0), (300, 8000, 800)]:
        L = T * 200
        b, s = ctypes.c_int(), ctypes.c_int()
        assert lib.wrnn_fold_shape(T, 200, 1, tgt, ovl, ctypes.byref(b), ctypes.byref(s)) == 0
        folded = OracleWaveRNN.fold_with_overlap(OracleWaveRNN, torch.zeros(1, L, 1), tgt, ovl)
        assert (b.value, s.value) == tuple(folded.shape[:2]), (T, tgt, ovl)
    assert lib.wrnn_fold_shape(10, 200, 0, 0, 0, ctypes.byref(b), ctypes.byref(s)) == 0
    assert (b.value, s.value) == (1, 2000)


def test_invalid_arguments_are_reported_not_crashed():
    from wavernn_amd import _abi
    lib = _abi.load_library()
    b, s = ctypes.c_int(), ctypes.c_int()
    assert lib.wrnn_fold_shape(0, 200, 1, 100, 10, ctypes.byref(b), ctypes.byref(s)) == _abi.WRNN_ERR_INVALID
    assert b'bad length' in lib.wrnn_last_error()
    cfg = _abi.WrnnConfig()
    cfg.model_type = 7
    h = ctypes.c_void_p()
    assert lib.wrnn_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == _abi.WRNN_ERR_INVALID
    cfg.model_type, cfg.mode, cfg.bits = 0, 0, 9
    cfg.n_upsample, cfg.hop_length = 3, 200
    for i, f in enumerate((5, 5, 7)):
        cfg.upsample_factors[i] = f
    cfg.res_out_dims = 128
    assert lib.wrnn_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == _abi.WRNN_ERR_INVALID
    assert b'hop_length' in lib.wrnn_last_error()


def test_product_fails_loudly_without_library(tmp_path):
    from wavernn_amd import _abi
    with pytest.raises(_abi.NativeLibraryMissing):
        _abi.load_library(str(tmp_path / 'missing.so'))


def test_beta_contract_host_restatement_matches_oracle():
    """wrnn_debug_beta evaluates csrc/philox.h beta_sample (the code the kernels run) on the
    host; it must agree with oracle/philox.py beta_sample for shapes below and above 1."""
    from oracle import philox
    from wavernn_amd import _abi
    lib = _abi.load_library()
    rng = np.random.default_rng(3)
    out = ctypes.c_float()
    for i in range(300):
        a, b = np.exp(rng.uniform(-3, 4, 2)).astype(np.float32)
        seed, stream, step, row = int(rng.integers(0, 2 ** 63)), i % 5, 17 * i, i % 7
        assert lib.wrnn_debug_beta(seed, stream, step, row, float(a), float(b),
                                   ctypes.byref(out)) == 0
        ref = philox.beta_sample(seed, stream, step, [row], np.float32([a]), np.float32([b]))[0]
        assert abs(out.value - float(ref)) <= 2e-6, (a, b, out.value, ref)
    assert lib.wrnn_debug_beta(0, 0, 0, 0, 0.0, 1.0, ctypes.byref(out)) == _abi.WRNN_ERR_INVALID


def test_beta_mode_is_geneing_only():
    from wavernn_amd import _abi
    lib = _abi.load_library()
    cfg = _abi.WrnnConfig()
    cfg.model_type, cfg.mode = _abi.WRNN_MODEL_FATCHORD, _abi.WRNN_MODE_BETA
    h = ctypes.c_void_p()
    assert lib.wrnn_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == _abi.WRNN_ERR_INVALID
    assert b'geneing' in lib.wrnn_last_error()


def test_wide_exchange_layout_exhaustive():
    """csrc/wide_layout.h, checked by the library's own host code for every row count of a wide
    group: each producer packet of a hop lands on exactly the consumer packet that expects its
    (row, unit quad), aligned, inside its slot; no-packet offsets fail the range check
    (the round-3 18-row deadlock)."""
    from wavernn_amd import _abi
    lib = _abi.load_library()
    assert [lib.wrnn_debug_wide_layout(r) for r in range(1, 17)] == [0] * 16
    assert lib.wrnn_debug_wide_layout(0) == _abi.WRNN_ERR_INVALID
    assert lib.wrnn_debug_wide_layout(17) == _abi.WRNN_ERR_INVALID


def test_fold_range_arguments_are_checked_on_the_host():
    """wrnn_set_fold_ranges (the single-utterance fold split): a null handle is
    refused with WRNN_ERR_INVALID without a device (ranges outside the folds, a count that does not
    match the call and wrnn_generate's refusal: tests/test_gpu_fold_split.py)."""
    from wavernn_amd import _abi
    lib = _abi.load_library()
    lo, hi = (ctypes.c_int * 1)(0), (ctypes.c_int * 1)(9)
    assert lib.wrnn_set_fold_ranges(None, lo, hi, 1) == _abi.WRNN_ERR_INVALID
    assert b'null handle' in lib.wrnn_last_error()
    assert lib.wrnn_set_utt_streams(None, None, 0) == _abi.WRNN_ERR_INVALID
