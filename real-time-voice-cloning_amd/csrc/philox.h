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

// MOL: torch uniform_(1e-5, 1 - 1e-5) restated on a 24-bit draw (oracle/philox.py mol_uniforms)
__host__ __device__ inline float mol_uniform_from_u32(uint32_t x) {
    const double U = (double)(x >> 8) * (1.0 / 16777216.0);
    const double lo = 1e-5, hi = 1.0 - 1e-5;
    return (float)(lo + (hi - lo) * U);
}

constexpr uint32_t kMolDomain = 0x80000000u;

}  // namespace wrnn
