"""Launch planner rates (runtime.hip plan_call): host only, through
wrnn_debug_plan (the plan wrnn_generate makes, every variant spill-free) and a rate table.

The planner minimises the summed per-step cost of its launches under a table of measured rates
(built-in defaults, or a per-build rates_mi355x.txt / WRNN_RATES file): C2 (18 rows) is three
rotated register-resident launches and C4 (144 rows) eleven time-sliced wide launches under the
defaults; perturbed tables must move the plan the way the costs say."""
import ctypes

import pytest

FAT, RR, GEN = 0, 1, 2
RAW, MOL = 0, 1
RING, WIDE, SPARSE, FORCE_SP = 2, 4, 1, 8


def plan(rows, S=12100, table=None, model=FAT, bits=9, mode=RAW, flags=RING | WIDE):
    from wavernn_amd import _abi
    lib = _abi.load_library()
    n, rot = ctypes.c_int(), ctypes.c_int()
    cap = 128
    nr, wd = (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
    rc = lib.wrnn_debug_plan(table.encode() if table else None, model, bits, mode, rows, S, flags,
                             ctypes.byref(n), nr, wd, cap, ctypes.byref(rot))
    if rc:
        raise ValueError(_abi.last_error())
    return [(nr[i], bool(wd[i])) for i in range(n.value)], rot.value


def test_default_rates_c2_is_three_rotated_launches():
    p, rot = plan(18)
    assert p == [(3, False)] * 3 and rot == 3


def test_default_rates_c4_is_eleven_time_sliced_wide_launches():
    p, rot = plan(144)
    assert p == [(16, True)] * 10 + [(2, True)] and rot == 0


def test_default_rates_fatchord_10bit_single_utterance_is_one_wide_launch():
    """The fork's fatchord default (10 bits, 3000 / 1500): 45 rows x 6,000 steps -- one wide
    launch of 6 rows per group (10.6 us per step measured, against 13.0 for two launches of 3
    rows per group; profiles/r06/b)."""
    p, rot = plan(45, S=6000, bits=10)
    assert p == [(6, True)] and rot == 0


def test_perturbed_register_rate_moves_the_plan():
    """3 rows per group made expensive: C2 takes one launch of 4 rows per group instead (and no
    rotation: its body is ceil(18 / 8) = 3 rows)."""
    p, rot = plan(18, table='fat9 4.8 5.15 50 6.92')
    assert p == [(4, False)] and rot == 0


def test_perturbed_wide_rate_moves_the_plan():
    p, _ = plan(18, table='wide 1.0 0.01 1.0')
    assert p == [(3, True)]


def test_perturbed_slice_threshold_keeps_the_unsliced_plan():
    p, _ = plan(144, table='slice 60 0.5')
    assert sorted(p) == [(2, False), (16, True)]


def test_sparse_family_chosen_by_rates():
    """Pruned weights (sparse image): the dense family wins under the measured rates (the sparse
    instances are slower on MI355X, §3.0g); cheap sparse rates or WRNN_SPARSE=1 pick them."""
    dense, _ = plan(18, flags=RING | WIDE | SPARSE)
    assert dense == [(3, False)] * 3
    assert plan(18, flags=RING | WIDE | SPARSE | FORCE_SP)[0] == [(3, False)] * 3
    cheap = 'fat9_sp 1 1.1 1.2 1.3\nrot9_sp 1 1.1 1.2 1.3'
    p, rot = plan(18, table=cheap, flags=RING | WIDE | SPARSE)
    assert p == [(3, False)] * 3 and rot == 3  # (the sparse rotated launches)
    p, _ = plan(30, table=cheap, flags=RING | WIDE | SPARSE)
    assert p == [(4, False)]


def test_runtimeracer_and_geneing_plans():
    assert plan(18, model=RR)[0] == [(3, False)] * 3
    assert plan(18, model=GEN, bits=10)[0] == [(3, False)] * 3
    assert plan(232, S=8000, model=RR, bits=10)[0] == [(16, True)] * 29


@pytest.mark.parametrize('table', ['nosuchkey 1 2', 'fat9 1 2 3', 'fat9 1 2 3 x', 'wide 1 -2 3'])
def test_bad_tables_are_refused(table):
    with pytest.raises(ValueError):
        plan(18, table=table)


def test_comments_and_blank_lines():
    p, _ = plan(18, table='# a comment\n\nfat9 4.8 5.15 50 6.92  # 3 rows made slow\n')
    assert p == [(4, False)]
