"""Near-tie analysis of a label difference between the HIP path and the reference (a helper of
the -m gpu parity tests, not a test module; the method of tools/near_tie_gpu.py).

Fold rows are independent recurrences, so each row's FIRST differing step is analysed on its
own: up to that step the row's labels equal the reference's, so the kernels' logits recorded
there (wrnn_set_debug_steps) are teacher-forced by the reference's history and comparable with
the oracle's logits at the same step. A difference is a near-tie when
  * the kernel's label is the exact decision on the kernel's OWN logits (wrnn_debug_decide:
    the kernels implement csrc/cand_key.h exactly), and
  * the oracle's margin between its label and the kernel's, v(k_ref) - v(k_gpu) with
    v = l + G formed exactly on the ORACLE's logits, is at most 2 x the kernel's logit error on
    those two classes plus the reference's own fp32 rounding of the decision (eps_ref).
Anything else is a real parity failure (an operation or a decision that differs).
"""
import numpy as np

from test_decision import decide, eps_ref


def first_divergence_per_row(a, b):
    out = []
    for r in range(a.shape[0]):
        d = np.nonzero(a[r] != b[r])[0]
        out.append(int(d[0]) if len(d) else -1)
    return np.array(out)


def exact_v(logits, seed, stream, step, fold):
    """float64 l + G of every class (G on its 2^-27 grid, philox.h gumbel_q_of: exact sum)."""
    from oracle import philox
    q = philox.raw_exp_noise(seed, stream, [step], [fold], len(logits))[0, 0].astype(np.float64)
    G = np.rint((-np.log(q) + 4.0) * 2.0 ** 27) * 2.0 ** -27 - 4.0
    return logits.astype(np.float64) + G


def divergence_steps(fd, limit=8):
    """The (at most `limit`, earliest) distinct first-divergence steps to record."""
    return sorted({int(s) for s in fd if s >= 0})[:limit]


def analyse(lib, seed, stream, gpu_labels, ref_labels, g_logits, o_logits, fold0=0):
    """Records of every row whose first divergence is at a step present in g_logits / o_logits
    ({step: (rows, n_classes)} of this utterance's rows). Each record carries `near_tie`."""
    fd = first_divergence_per_row(gpu_labels, ref_labels)
    recs = []
    for row in np.flatnonzero(fd >= 0):
        step = int(fd[row])
        if step not in g_logits:
            continue
        g, o = g_logits[step][row], o_logits[step][row]
        kg, ko = int(gpu_labels[row, step]), int(ref_labels[row, step])
        exact_label = decide(lib, seed, stream, step, fold0 + int(row), g)[0]
        v = exact_v(o, seed, stream, step, fold0 + int(row))
        margin = float(v[ko] - v[kg])
        err = float(max(abs(float(g[ko]) - float(o[ko])), abs(float(g[kg]) - float(o[kg]))))
        bound = 2 * err + float(eps_ref(o[ko], o[kg], o.max()))
        recs.append(dict(row=int(row), step=step, gpu_label=kg, ref_label=ko, gpu_exact_label=exact_label,
                         ref_margin=margin, logit_err=err, bound=bound, max_abs_logit=float(np.abs(o).max()),
                         near_tie=bool(exact_label == kg and margin <= bound)))
    return fd, recs
