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
