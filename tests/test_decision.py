"""The RAW sampling decision of every kernel (csrc/cand_key.h), checked on the host
through wrnn_debug_decide -- the same C++ the kernels compile -- without a GPU:

* against the REAL reference: at every step where tests/golden holds the reference's own logits
  (fatchord_version.py:213 / runtimeracer_version.py:270, captured by gen_golden.py), the exact
  decision argmax_k (l_k + G_k) on those logits must equal the label the reference drew
  (fatchord_version.py:224-228: softmax -> Categorical), unless the reference's own fp32 rounding
  could have decided it (a top-2 margin below EPS_REF);
* against float64 ground truth: the two-word key orders l + G exactly as float64 does (l fp32,
  G on its 2^-27 grid: the sum is exact in float64), ties to the lowest class, including
  adversarial near-ties built a few ulps apart;
* the fixed-point noise word against numpy's float64 -log(q) of the oracle's q.
"""
import ctypes
import json
import os

import numpy as np

from conftest import REPO

# The reference's own rounding of its decision, in the log domain: per class exp (<= 1 ulp),
# three divisions (probs / sum, / sum again, / q: 0.5 ulp each) -> 2.5 ulp = 5 u relative per
# side, u = 2^-24, both sides 10 u; plus the fp32 rounding of l - max(l) (0.5 ulp(|l - max|) per
# side). A decision whose exact margin is below this can go either way in fp32.
U = 2.0 ** -24


def eps_ref(l1, l2, lmax):
    return 10 * U + 0.5 * (np.spacing(np.float32(abs(l1 - lmax))) + np.spacing(np.float32(abs(l2 - lmax))))


def lib():
    from wavernn_amd import _abi
    return _abi.load_library()


def decide(L, seed, stream, step, fold, logits):
    lab, margin = ctypes.c_int(), ctypes.c_double()
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    rc = L.wrnn_debug_decide(seed, stream, step, fold, lg.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                             len(lg), ctypes.byref(lab), ctypes.byref(margin))
    assert rc == 0
    return lab.value, margin.value


def gumbel_q(seed, stream, steps, rows, n):
    """numpy restatement of philox.h gumbel_q_of over the oracle's fp32 q."""
    from oracle import philox
    q = philox.raw_exp_noise(seed, stream, steps, rows, n).astype(np.float64)
    return np.rint((-np.log(q) + 4.0) * 2.0 ** 27).astype(np.int64)


def test_noise_word_is_the_fixed_point_gumbel_of_the_oracle_q():
    from oracle import philox
    seed, stream = 12345, 3
    gq = gumbel_q(seed, stream, [0, 7, 4000], [0, 5], 512)
    assert gq.min() > 0 and gq.max() < 2 ** 32
    G = gq * 2.0 ** -27 - 4.0
    q = philox.raw_exp_noise(seed, stream, [0, 7, 4000], [0, 5], 512).astype(np.float64)
    assert np.max(np.abs(G + np.log(q))) <= 2.0 ** -28 + 1e-15
    # the host decision sees exactly these words: a one-hot logit spike far above the noise range
    # must win, and with equal logits the decision is argmax G (lowest class on a tie)
    L = lib()
    for step, row in ((0, 0), (7, 5), (4000, 0)):
        lg = np.zeros(512, np.float32)
        lab, _ = decide(L, seed, stream, step, row, lg)
        g = gq[[0, 7, 4000].index(step), [0, 5].index(row)]
        assert lab == int(np.flatnonzero(g == g.max())[0])
        lg[311] = 100.0
        assert decide(L, seed, stream, step, row, lg)[0] == 311


def test_key_orders_exactly_like_float64():
    """Random logits, plus adversarial near-ties: a class placed 0, 1, 2, 3 ulps (of l + G) and a
    few 2^-27 grid steps from the best one. The key's decision must be float64's argmax of the
    exact l + G with ties to the lowest class, wherever the top-2 margin exceeds the key's
    resolution (2^-29 |v|)."""
    L = lib()
    rng = np.random.default_rng(5)
    checked = near = 0
    for it in range(400):
        n = int(rng.choice([30, 256, 512, 1024]))
        n -= n % 4
        seed, stream, step, fold = int(rng.integers(0, 2 ** 63)), it % 3, int(rng.integers(0, 12100)), it % 18
        scale = float(rng.choice([0.2, 3.0, 20.0, 40.0]))
        lg = (rng.standard_normal(n) * scale).astype(np.float32)
        gq = gumbel_q(seed, stream, [step], [fold], n)[0, 0]
        G = gq * 2.0 ** -27 - 4.0
        v = lg.astype(np.float64) + G
        if it % 2:  # make a near-tie with the current best: l_j chosen so v_j ~ v_best + d
            b = int(np.argmax(v))
            j = int(rng.integers(0, n))
            if j != b:
                d = float(rng.choice([0.0, 1.0, -1.0, 2.0, 3.0])) * np.spacing(np.float32(abs(v[b]) + 1e-30))
                lg[j] = np.float32(v[b] + d - G[j])
                v = lg.astype(np.float64) + G
                near += 1
        top = np.sort(v)[-2:]
        lab, margin = decide(L, seed, stream, step, fold, lg)
        assert abs(margin - (top[1] - top[0])) <= 1e-12 * max(1.0, abs(top[1]))
        if top[1] - top[0] > 2.0 ** -29 * abs(top[1]):
            assert lab == int(np.argmax(v)), (it, lab, int(np.argmax(v)), top)
            checked += 1
        else:  # a tie at the key's resolution: one of the tied classes, the lowest on an exact tie
            tied = np.flatnonzero(v >= top[1] - 2.0 ** -29 * abs(top[1]))
            assert lab in tied
            if top[1] == top[0]:
                assert lab == int(tied[0])
    assert checked > 300 and near > 150


def test_exact_decision_reproduces_every_reference_label_it_can():
    """Every recorded (step, row) of every RAW/BITS golden fixture: the exact decision on the
    REFERENCE's logits equals the reference's label wherever the margin exceeds the reference's
    own rounding; the few below it are counted (none expected on these fixtures)."""
    L = lib()
    meta = json.load(open(os.path.join(REPO, 'tests', 'golden', 'golden_meta.json')))
    total = ambiguous = 0
    for name, m in meta.items():
        path = os.path.join(REPO, 'tests', 'golden', name + '.npz')
        if name.startswith('_') or not os.path.exists(path) or m['mode'] not in ('RAW', 'BITS'):
            continue
        g = np.load(path)
        if 'labels' not in g.files:
            continue  # geneing RAW = Beta
        for i, step in enumerate(g['logits_steps']):
            for row in range(g['logits'].shape[1]):
                lg = g['logits'][i, row]
                lab, margin = decide(L, int(m['noise_seed']), int(m['stream']), int(step), row, lg)
                ref = int(g['labels'][row, step])
                total += 1
                if lab != ref:
                    gq = gumbel_q(int(m['noise_seed']), int(m['stream']), [int(step)], [row], len(lg))[0, 0]
                    v = lg.astype(np.float64) + (gq * 2.0 ** -27 - 4.0)
                    e = eps_ref(lg[lab], lg[ref], lg.max())
                    assert v[lab] - v[ref] <= e, (name, step, row, lab, ref, v[lab] - v[ref], e)
                    ambiguous += 1
    assert total > 400
    assert ambiguous == 0, ambiguous


def test_decide_rejects_bad_arguments():
    from wavernn_amd import _abi
    L = lib()
    lab = ctypes.c_int()
    lg = np.zeros(8, np.float32)
    p = lg.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert L.wrnn_debug_decide(0, 0, 0, 0, p, 1, ctypes.byref(lab), None) == _abi.WRNN_ERR_INVALID
    assert L.wrnn_debug_decide(0, 0, 0, 0, None, 8, ctypes.byref(lab), None) == _abi.WRNN_ERR_INVALID
    assert L.wrnn_debug_decide(0, 0, 0, 0, p, 8, ctypes.byref(lab), None) == 0
