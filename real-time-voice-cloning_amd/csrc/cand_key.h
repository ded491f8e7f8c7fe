// The sampler's decision key (RAW categorical), shared by every kernel that samples: the
// persistent kernels (kernels_persist*.hip, through persist_common.h) and the CHAIN engine's
// k_sample (kernels_step.hip). Host-callable too (wrnn_debug_cand_key checks it on the CPU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox.h"

namespace wrnn {

// ---- the sampler's decision: a two-word key per (row, class) ------------------------------
// The reference decides k* = argmax_k (softmax(l)_k / sum) / q_k in fp32
// (fatchord_version.py:224-228, runtimeracer_version.py:280-281: Categorical.sample() is
// torch.multinomial's argmax(p / q) fast path). In exact arithmetic that is
// argmax_k (l_k + G_k), G_k = -log q_k. Round 4 evaluated l + g in fp32 with g = -logf(q): an
// absolute rounding of ~ulp(|l + g|) + ulp(|g|), up to ~1e-6 at |l + g| ~ 8 -- more than the
// reference's own fp32 p / q rounding, and one measured flip came from exactly that (VERDICT r4
// Missing #1). Now G comes in fixed point to 2^-27 (philox.h gumbel_q_of: float64 logs, error
// <= 3.7e-9) and v = l + G is formed EXACTLY as an unevaluated fp32 pair (s, r), v = s + r,
// |r| <= ulp(s) / 2 (TwoSum, then Fast2Sum; no float64 -- its register pairs spilled the
// kernels at 255 VGPRs): given the logits the decision's only error is G's quantisation, below
// the reference's own fp32 rounding, so the kernels can differ from the reference only where the
// REFERENCE's rounding decides.
// Key = (hi, lo), compared lexicographically as unsigned words (the same three compares and two
// selects per step as round 4's (value, class) argmax): hi = the order-preserving image of s
// (sign flip), lo = the top 13 bits of the order-preserving image of r, then 12 bits of
// (4095 - class), then the 7-bit exchange tag. Equal hi means equal s, so the order of lo is
// the order of v; r keeps 4 mantissa bits, so v is resolved to |r| / 16 <= ulp(s) / 32 (2^-29
// relative, 3e-8 at |v| = 16 -- 5x below the reference's own fp32 rounding) and candidates
// closer than that count as ties. The max key is the argmax of v with ties to the lowest class
// (torch.argmax's first maximum). A lane without a class contributes (0, 0), below every real
// key.
struct CandKey {
    uint32_t hi, lo;
};
__host__ __device__ __forceinline__ uint32_t f32_order(float f) {
    const uint32_t b = __builtin_bit_cast(uint32_t, f);
    return (b >> 31) ? ~b : (b | 0x80000000u);
}
__host__ __device__ __forceinline__ CandKey cand_key(float l, uint32_t gq, int cls) {
#pragma clang fp contract(off)
    // G = ga + gb exactly: (gq >> 8) 2^-19 - 4 is on a 2^-19 grid below 32 in magnitude (24 bits)
    const float ga = (float)(gq >> 8) * 0x1p-19f - 4.0f;
    const float gb = (float)(gq & 0xffu) * 0x1p-27f;
    const float s = l + ga;  // TwoSum(l, ga): s + e == l + ga exactly
    const float bp = s - l;
    const float e = (l - (s - bp)) + (ga - bp);
    const float r = e + gb;  // |e| <= ulp(s) / 2, gb < 2^-19: rounding ~2^-43, immaterial
    const float s2 = s + r;  // Fast2Sum(s, r): s2 + r2 == s + r, |r2| <= ulp(s2) / 2
    const float r2 = r - (s2 - s);
    return CandKey{f32_order(s2), (f32_order(r2) & 0xfff80000u) | (uint32_t)(0xfff - cls) << 7};
}
__host__ __device__ __forceinline__ int key_cls(uint32_t lo) { return 0xfff - (int)((lo >> 7) & 0xfffu); }
// exchange tag of step seq in the key's low 7 bits: never 0, so a cleared candidate slot never
// reads as ready; 6 bits of the step suffice (a slot holds step t - 1's or step t's key)
constexpr uint32_t kKeyTagMask = 0x7fu;
__host__ __device__ __forceinline__ unsigned key_tag(unsigned seq) { return 0x40u | (seq & 0x3fu); }

// (h, l) <- (h2, l2) when that key is larger (bitwise, as amax_take)
__device__ __forceinline__ void kmax_take(uint32_t& h, uint32_t& l, uint32_t h2, uint32_t l2) {
    const bool take = (h2 > h) | ((h2 == h) & (l2 > l));
    h = take ? h2 : h;
    l = take ? l2 : l;
}
template <int CTRL>
__device__ __forceinline__ void kmax_dpp_step(uint32_t& h, uint32_t& l) {
    const uint32_t h2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)h, CTRL, 0xf, 0xf, false);
    const uint32_t l2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)l, CTRL, 0xf, 0xf, false);
    kmax_take(h, l, h2, l2);
}
// max key over the 16 lanes of a DPP row; every lane of the row receives it
__device__ __forceinline__ void row16_kmax(uint32_t& h, uint32_t& l) {
    kmax_dpp_step<0xB1>(h, l);
    kmax_dpp_step<0x4E>(h, l);
    kmax_dpp_step<0x124>(h, l);
    kmax_dpp_step<0x128>(h, l);
}
// max key over the 32 lanes of a half-wave, valid in its upper 16 lanes (as half_argmax)
__device__ __forceinline__ void half_kmax(uint32_t& h, uint32_t& l) {
    row16_kmax(h, l);
    const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp((int)h, (int)h, 0x142, 0xA, 0xF, false);
    const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp((int)l, (int)l, 0x142, 0xA, 0xF, false);
    kmax_take(h, l, h2, l2);
}

}  // namespace wrnn
