"""Row rotation of the persistent engine (runtime.hip plan_rotation), host
planner only: wrnn_debug_rot_plan without a device.

For R fold rows on the 8 XCD groups (q = R // 8, m = R % 8 groups of q + 1 rows), the plan's K
launches must put every row in exactly one slot of every launch (a group of q + 1 rows uses all
its slots, a group of q rows leaves its last one empty), advance each row's step offset by the
steps its group ran, bring every row to exactly S steps, keep the groups' wall times balanced
(n_hi t(q + 1) ~ n_lo t(q)) and beat the single launch at t(q + 1)."""
import ctypes

import numpy as np
import pytest

US = {1: 4.8, 2: 5.22, 3: 5.91}  # (the runtime's rates; 2 rows: the rotated instance's)


def plan(R, S=12100):
    from wavernn_amd import _abi
    lib = _abi.load_library()
    k, nh, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    q = R // 8
    cap = 24 * 8 * (q + 1) * 2
    vm = (ctypes.c_int * cap)()
    assert lib.wrnn_debug_rot_plan(R, S, US[q + 1], US[q], ctypes.byref(k), ctypes.byref(nh), ctypes.byref(nl),
                                   vm, cap) == 0
    K = k.value
    return K, nh.value, nl.value, np.array(vm[:K * 8 * (q + 1) * 2]).reshape(K, q + 1, 8, 2)


@pytest.mark.parametrize('R', [9, 10, 12, 17, 18, 20])
def test_rotation_plan_invariants(R):
    S = 12100
    K, nh, nl, vm = plan(R, S)
    assert K > 1
    q, m = R // 8, R % 8
    off = np.zeros(R, int)
    for j in range(K):
        seen = []
        for g in range(8):
            nr = q + 1 if g < m else q
            for r in range(q + 1):
                row, o = vm[j, r, g]
                if r >= nr:
                    assert (row, o) == (-1, -1)
                    continue
                assert 0 <= row < R and o == off[row], (j, g, r, row, o, off[row])
                seen.append((row, nr))
        assert sorted(x[0] for x in seen) == list(range(R)), f'launch {j}: every row once'
        for row, nr in seen:
            off[row] += nh if nr == q + 1 else nl
    assert (off == S).all()
    # balanced wall time per launch, and a gain over the single launch at t(q + 1)
    t_hi, t_lo = US[q + 1], US[q]
    assert abs(nh * t_hi - nl * t_lo) <= 0.02 * max(nh * t_hi, nl * t_lo)  # (integer steps)
    assert K * max(nh * t_hi, nl * t_lo) < 0.98 * S * t_hi
    # C2 (18 rows): three launches of 3706 steps at 3 rows / 4197 at 2
    if R == 18:
        assert (K, nh, nl) == (3, 3706, 4197)


@pytest.mark.parametrize('R', [8, 16, 24, 7, 23, 31, 40])
def test_no_rotation_where_it_cannot_pay(R):
    """Even groups (R % 8 == 0), single-row groups only (R < 8), 4-row groups (no spill-free
    rotated instance) and near-full groups (too many launches for the gain) keep one launch."""
    from wavernn_amd import _abi
    lib = _abi.load_library()
    k, nh, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    q = R // 8
    t_hi, t_lo = US.get(q + 1, 6.92), US.get(q, 4.8)
    assert lib.wrnn_debug_rot_plan(R, 12100, t_hi, t_lo, ctypes.byref(k), ctypes.byref(nh), ctypes.byref(nl),
                                   None, 0) == 0
    assert k.value == 0


def slice_plan(R, S=12100):
    from wavernn_amd import _abi
    lib = _abi.load_library()
    k = ctypes.c_int()
    rs = (ctypes.c_int * 128)()
    vm = (ctypes.c_int * (64 * 128 * 2))()
    assert lib.wrnn_debug_slice_plan(R, S, ctypes.byref(k), rs, 128, vm, 64 * 128 * 2) == 0
    K = k.value
    return K, np.array(rs[:2 * K]).reshape(K, 2), np.array(vm[:K * 128 * 2]).reshape(K, 16, 8, 2)


@pytest.mark.parametrize('R', [136, 144, 160, 192, 264, 360])
def test_wide_time_slices_plan_invariants(R):
    """Time-sliced wide launches: at most 16 rows per group and launch, every
    row at most once per launch and in its own group (rows g + 8 i), offsets advanced by the
    launch's steps, every row at exactly S. C4 (144 rows): 9 launches of 1,512 steps at 16 rows
    per group, then 2 of the remaining 4 steps (16 and 2 rows per group)."""
    S = 12100 if R < 300 else 6000
    K, rs, vm = slice_plan(R, S)
    assert K > 1
    off = np.zeros(R, int)
    for k in range(K):
        nr, steps = rs[k]
        assert 1 <= nr <= 16 and steps >= 1
        rows = []
        for g in range(8):
            for r in range(16):
                row, o = vm[k, r, g]
                if r >= nr:
                    assert (row, o) == (-1, -1)
                    continue
                assert row % 8 == g and o == off[row], (k, g, r, row, o, off[row])
                rows.append(row)
        assert len(rows) == len(set(rows)) == 8 * nr
        off[rows] += steps
    assert (off == S).all()
    if R == 144:
        assert K == 11 and rs[:9].tolist() == [[16, 1512]] * 9 and rs[9:].tolist() == [[16, 4], [2, 4]]


@pytest.mark.parametrize('R', [128, 120, 143, 256, 384, 18])
def test_wide_time_slices_only_above_16_rows_per_group_and_off_multiples_of_16(R):
    assert slice_plan(R)[0] == 0
