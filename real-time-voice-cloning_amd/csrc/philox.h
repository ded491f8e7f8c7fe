// Philox4x32-10 (Salmon, Moraes, Dror, Shaw; SC'11) -- the noise contract of the sampler.
// Bit-identical to the oracle's numpy restatement (oracle/philox.py); checked against the
// Random123 known-answer vectors in tests/test_philox.py (host) and on the GPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wrnn {

struct U4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                             uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return U4{c0, c1, c2, c3};
}

// RAW: Exp(1) variate from one 32-bit word (oracle/philox.py raw_exp_noise)
__host__ __device__ inline float exp1_from_u32(uint32_t x) {
    const double u = (2.0 * (double)(x >> 9) + 1.0) * (1.0 / 16777216.0);
    return (float)(-log(u));
}

// RAW Gumbel noise g = -log(q), q the contract's Exp(1) variate (philox.h exp1_from_u32, its
// float64 log kept exact): argmax_k (l_k + g_k) is the decision of argmax_k ((softmax(l)_k / sum)
// / q_k). The second log runs in fp32 (logf, ~1 ulp: the order of the fp32 rounding the
// reference's own p / q carries; both logs in float64 took 0.88 instead of 0.54 ms per C2 call,
// labels unchanged).
__host__ __device__ inline float gumbel_of(uint32_t x) {
    return -logf(exp1_from_u32(x));
}
// The sampler's noise since round 5: G = -log q of the same fp32 q (the reference's q tensor is
// fp32), taken in float64 and stored as a 32-bit fixed-point word, (G + 4) * 2^27 rounded to the
// nearest integer: q lies in [5.96e-8, 16.64], so G + 4 in [1.19, 20.64] and the word < 2^32;
// the quantisation error is <= 2^-28 = 3.7e-9 absolute -- below even the last fp32 division of
// the reference's own p / q (2^-24 relative) -- and the noise still costs 4 bytes per class.
// cand_key.h adds it to the fp32 logit exactly, as an fp32 pair (TwoSum, then Fast2Sum).
constexpr double kGumbelOffset = 4.0;
constexpr double kGumbelScale = 134217728.0;  // 2^27
__host__ __device__ inline uint32_t gumbel_q_of(uint32_t x) {
    const double G = -log((double)exp1_from_u32(x));
    return (uint32_t)rint((G + kGumbelOffset) * kGumbelScale);
}

// MOL: torch uniform_(1e-5, 1 - 1e-5) restated on a 24-bit draw (oracle/philox.py mol_uniforms)
__host__ __device__ inline float mol_uniform_from_u32(uint32_t x) {
    const double U = (double)(x >> 8) * (1.0 / 16777216.0);
    const double lo = 1e-5, hi = 1.0 - 1e-5;
    return (float)(lo + (hi - lo) * U);
}

constexpr uint32_t kMolDomain = 0x80000000u;

// BETA: geneing 'RAW' mode (vocoder/distribution.py:7-20, Beta(exp(l0), exp(l1)).sample()) on
// the stream: X / (X + Y) with X ~ Gamma(alpha), Y ~ Gamma(beta) by Marsaglia-Tsang in float64
// (oracle/philox.py gamma_mt / beta_sample, same operation order, contraction off).
constexpr uint32_t kBetaDomain = 0x40000000u;
constexpr int kBetaTries = 16;

__host__ __device__ inline double u_open_from_u32(uint32_t x) {
    return (2.0 * (double)(x >> 9) + 1.0) * (1.0 / 16777216.0);
}

__host__ __device__ inline double gamma_mt(double a, uint32_t g, uint32_t step, uint32_t row,
                                           uint32_t stream, uint32_t k0, uint32_t k1) {
#pragma clang fp contract(off)
    const bool boost = a < 1.0;
    const double ap = boost ? a + 1.0 : a;
    const double d = ap - 1.0 / 3.0;
    const double c = 1.0 / sqrt(9.0 * d);
    double out = d, ub = 1.0;
    for (int k = 0; k < kBetaTries; ++k) {
        const U4 w = philox4x32_10(kBetaDomain | (g << 8) | (uint32_t)k, step, row, stream, k0, k1);
        const double u0 = u_open_from_u32(w.x), u1 = u_open_from_u32(w.y);
        const double u2 = u_open_from_u32(w.z), u3 = u_open_from_u32(w.w);
        const double z = sqrt(-2.0 * log(u0)) * cos((2.0 * 3.141592653589793) * u1);
        const double t = 1.0 + c * z;
        const double v = (t * t) * t;
        if (v > 0.0) {
            const double rhs = ((0.5 * z) * z + d - d * v) + d * log(v);
            if (log(u2) < rhs) {
                out = d * v;
                ub = u3;
                break;
            }
        }
    }
    if (boost) out = out * pow(ub, 1.0 / a);
    const double tiny = 2.2250738585072014e-308;  // DBL_MIN
    return out > tiny ? out : tiny;
}

// Beta(alpha, beta) rescaled to [-1, 1] in float32 (the reference's 2.0 * sample - 1.0)
__host__ __device__ inline float beta_sample(float alpha, float beta, uint32_t step, uint32_t row,
                                             uint32_t stream, uint32_t k0, uint32_t k1) {
#pragma clang fp contract(off)
    const double x = gamma_mt((double)alpha, 0u, step, row, stream, k0, k1);
    const double y = gamma_mt((double)beta, 1u, step, row, stream, k0, k1);
    const float s = (float)(x / (x + y));
    return 2.0f * s - 1.0f;
}

}  // namespace wrnn
