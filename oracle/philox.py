"""Philox4x32-10 counter-based RNG and the noise contract of the WaveRNN sampler.

TEST INFRASTRUCTURE ONLY. This module belongs to the CPU oracle: only tests/,
tests/golden/gen_golden.py, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import it. The product path generates the same noise on the GPU in
real-time-voice-cloning_amd/csrc/philox.h and never imports this file.

Why injected noise
------------------
The reference samples with torch's global CPU generator:

* RAW mode, ``vocoder/models/fatchord_version.py:225-228`` (runtimeracer ``:280-283``):
  ``torch.distributions.Categorical(softmax(logits)).sample()``. In torch 2.10 that is
  ``multinomial(probs, 1)`` whose single-sample fast path computes
  ``argmax(probs / q)`` with ``q ~ Exp(1)`` drawn by ``Tensor.exponential_``.
* MOL mode, ``vocoder/distribution.py:123,135``: two ``Tensor.uniform_(1e-5, 1-1e-5)``
  draws per step, shape ``(1, B, 10)`` then ``(1, B)``.

torch's CPU stream cannot be reproduced on a GPU, so parity is defined on an injected
stream: both the reference (patched, see tests/golden/gen_golden.py) and the MI355X path
draw their noise from this Philox stream.

Contract (bit-for-bit identical to csrc/philox.h)
-------------------------------------------------
key  = (seed & 0xffffffff, seed >> 32)
RAW  : counter = (k >> 2, step, row, stream), word k & 3 of the output block
       u = (2 * (x >> 9) + 1) * 2**-24            (exact in f32, 0 < u < 1)
       q = float32(-log(float64(u)))              (Exp(1) variate)
MOL  : counter = (0x80000000 | j, step, row, stream) for j = 0, 1, 2 -> 12 words w[0..11]
       U = (w >> 8) * 2**-24
       u = float32(1e-5 + (1 - 1e-5 - 1e-5) * U)  (torch ``uniform_(1e-5, 1.0 - 1e-5)``)
       u1[m] = u(w[m]) for the 10 mixtures, u2 = u(w[10])
BETA : geneing 'RAW' mode, ``vocoder/distribution.py:7-20`` ``Beta(alpha, beta).sample()``
       (torch: Dirichlet over two standard gammas, rejection-sampled from the global generator)
       restated on the stream as X / (X + Y), X ~ Gamma(alpha), Y ~ Gamma(beta) by
       Marsaglia-Tsang (2000) in float64, gamma g = 0 (alpha) / 1 (beta), attempt k < 16:
       counter = (0x40000000 | g << 8 | k, step, row, stream) -> 4 words, u_i as RAW's u
       (open (0, 1)); a' = a + 1 if a < 1 else a; d = a' - 1/3; c = 1 / sqrt(9 d)
       z = sqrt(-2 log u0) * cos(2 pi u1); t = 1 + c z; v = (t t) t
       accept the first k with v > 0 and log u2 < ((0.5 z) z + d - d v) + d log v: G = d v
       (no accepted attempt: G = d); a < 1: G = G * u3 ** (1 / a) (u3 of the accepted attempt)
       G = max(G, DBL_MIN); sample = float32(X / (X + Y)); returned 2 sample - 1 in float32
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

MOL_DOMAIN = 0x80000000
MOL_LO = 1e-5
MOL_HI = 1.0 - 1e-5
BETA_DOMAIN = 0x40000000
BETA_TRIES = 16


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32 with 10 rounds (Salmon et al., SC'11).

    All arguments broadcast; returns four uint32 arrays.
    """
    c0 = np.asarray(c0, dtype=np.uint32)
    c1 = np.asarray(c1, dtype=np.uint32)
    c2 = np.asarray(c2, dtype=np.uint32)
    c3 = np.asarray(c3, dtype=np.uint32)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (a.astype(np.uint32) for a in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32


def raw_u32(seed, stream, steps, rows, n_classes):
    """Raw Philox words for RAW sampling: shape (len(steps), len(rows), n_classes)."""
    assert n_classes % 4 == 0
    k0, k1 = seed_key(seed)
    steps = np.asarray(steps, dtype=np.uint32)
    rows = np.asarray(rows, dtype=np.uint32)
    groups = np.arange(n_classes // 4, dtype=np.uint32)
    c0 = groups[None, None, :]
    c1 = steps[:, None, None]
    c2 = rows[None, :, None]
    out = philox4x32_10(c0, c1, c2, np.uint32(stream), k0, k1)
    w = np.stack(out, axis=-1)  # (S, B, n/4, 4)
    return w.reshape(len(steps), len(rows), n_classes)


def raw_exp_noise(seed, stream, steps, rows, n_classes):
    """Exp(1) noise q for RAW sampling, float32, shape (S, B, n_classes)."""
    x = raw_u32(seed, stream, steps, rows, n_classes)
    u = (2.0 * (x >> np.uint32(9)).astype(np.float64) + 1.0) * (2.0 ** -24)
    return (-np.log(u)).astype(np.float32)


def mol_uniforms(seed, stream, steps, rows):
    """(u1, u2) for MOL sampling: u1 (S, B, 10) float32, u2 (S, B) float32."""
    k0, k1 = seed_key(seed)
    steps = np.asarray(steps, dtype=np.uint32)
    rows = np.asarray(rows, dtype=np.uint32)
    words = []
    for j in range(3):
        out = philox4x32_10(np.uint32(MOL_DOMAIN | j), steps[:, None], rows[None, :],
                            np.uint32(stream), k0, k1)
        words.extend(out)
    w = np.stack(words, axis=-1)  # (S, B, 12)
    U = (w >> np.uint32(8)).astype(np.float64) * (2.0 ** -24)
    u = (MOL_LO + (MOL_HI - MOL_LO) * U).astype(np.float32)
    return u[..., :10].copy(), u[..., 10].copy()


def _u_open(x):
    """Open-interval uniform of a 32-bit word, as RAW's (2 (x >> 9) + 1) 2**-24, float64."""
    return (2.0 * (np.asarray(x, dtype=np.uint32) >> np.uint32(9)).astype(np.float64) + 1.0) * (2.0 ** -24)


def gamma_mt(seed, stream, step, rows, a, g):
    """Standard gamma variates (float64, shape (B,)) of shape a (float64 (B,)) for gamma index g
    (0 alpha, 1 beta) at one step -- Marsaglia-Tsang on the Philox stream (BETA contract)."""
    k0, k1 = seed_key(seed)
    rows = np.asarray(rows, dtype=np.uint32)
    a = np.asarray(a, dtype=np.float64)
    boost = a < 1.0
    ap = np.where(boost, a + 1.0, a)
    d = ap - 1.0 / 3.0
    c = 1.0 / np.sqrt(9.0 * d)
    out = d.copy()
    ub = np.ones_like(a)
    done = np.zeros(a.shape, dtype=bool)
    with np.errstate(invalid='ignore', divide='ignore'):
        for k in range(BETA_TRIES):
            w = philox4x32_10(np.uint32(BETA_DOMAIN | (g << 8) | k), np.uint32(step), rows,
                              np.uint32(stream), k0, k1)
            u0, u1, u2, u3 = (_u_open(x) for x in w)
            z = np.sqrt(-2.0 * np.log(u0)) * np.cos(2.0 * np.pi * u1)
            t = 1.0 + c * z
            v = (t * t) * t
            vpos = v > 0.0
            rhs = ((0.5 * z) * z + d - d * v) + d * np.log(np.where(vpos, v, 1.0))
            take = vpos & (np.log(u2) < rhs) & ~done
            out = np.where(take, d * v, out)
            ub = np.where(take, u3, ub)
            done |= take
    out = np.where(boost, out * np.power(ub, 1.0 / a), out)
    return np.maximum(out, np.finfo(np.float64).tiny)


def beta_sample(seed, stream, step, rows, alpha, beta):
    """Beta(alpha, beta) rescaled to [-1, 1] (float32, shape (B,)) -- the BETA contract.
    alpha, beta: float32 arrays (exp of the two fc3 outputs, vocoder/distribution.py:14-16)."""
    x = gamma_mt(seed, stream, step, rows, np.asarray(alpha, np.float32).astype(np.float64), 0)
    y = gamma_mt(seed, stream, step, rows, np.asarray(beta, np.float32).astype(np.float64), 1)
    s = (x / (x + y)).astype(np.float32)
    return np.float32(2.0) * s - np.float32(1.0)
