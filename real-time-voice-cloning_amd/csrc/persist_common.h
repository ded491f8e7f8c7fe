// Device helpers shared by the persistent recurrence kernels (kernels_persist.hip: fatchord,
// kernels_persist_rr.hip: runtimeracer): timers, DPP reductions, gate nonlinearities, buffer
// resource access, tagged-pair exchanges over the XCD-shared L2.
#pragma once
#include <cstdlib>
#include <cstring>

#include "wrnn_kernels.h"
#include "cand_key.h"

namespace wrnn {

constexpr unsigned kSpinTicks = 100000000u;  // 1 s of s_memrealtime (100 MHz)

__device__ __forceinline__ unsigned p_now() { return (unsigned)__builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ unsigned ld_nt_u(const unsigned* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float ld_nt_f(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float4 ld_nt_f4(const float4* p) {
    const float* q = reinterpret_cast<const float*>(p);
    return make_float4(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1),
                       __builtin_nontemporal_load(q + 2), __builtin_nontemporal_load(q + 3));
}
__device__ __forceinline__ unsigned ld_sc1_u(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int CTRL>
__device__ __forceinline__ float pdpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
// sum over the 16 lanes of a DPP row; every lane of the row receives the same total
__device__ __forceinline__ float row16_sum(float v) {
    v += pdpp<0xB1>(v);   // quad_perm xor 1
    v += pdpp<0x4E>(v);   // quad_perm xor 2
    v += pdpp<0x124>(v);  // row_ror 4
    v += pdpp<0x128>(v);  // row_ror 8
    return v;
}

// Gate nonlinearities on the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32, ~1 ulp each):
// sigmoid(x) = 1 / (1 + 2^(-x log2 e)), tanh(x) = 1 - 2 / (2^(2x log2 e) + 1). Within a few ulp
// of torch's vectorised sigmoid / tanh -- the same order as the fp32 summation-order
// differences of the matrix products -- at a fraction of the cost of expf / IEEE division /
// tanhf; the RAW label parity tests run on this path.
__device__ __forceinline__ float p_sigmoid(float x) {
    const float e = __builtin_amdgcn_exp2f(-x * 1.4426950408889634f);
    return __builtin_amdgcn_rcpf(1.0f + e);
}
__device__ __forceinline__ float p_tanh(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
    return 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
}
// torch GRUCell gate arithmetic (same operation order as kernels_step.hip gru_cell)
__device__ __forceinline__ float p_gru(float gi_r, float gi_z, float gi_n, float gh_r, float gh_z,
                                       float gh_n, float h) {
#pragma clang fp contract(off)
    const float r = p_sigmoid(gh_r + gi_r);
    const float z = p_sigmoid(gh_z + gi_z);
    const float ghr = gh_n * r;
    const float n = p_tanh(gi_n + ghr);
    const float d = h - n;
    const float dz = d * z;
    return dz + n;
}
__device__ __forceinline__ float p_add(float a, float b) {
#pragma clang fp contract(off)
    return a + b;
}

// packed fp32 (v_pk_fma_f32): even/odd-k partial sums of one (output, row) dot product
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void dot4(v2f& acc, const float4 w, const float4 x) {
    acc = __builtin_elementwise_fma((v2f){w.x, w.y}, (v2f){x.x, x.y}, acc);
    acc = __builtin_elementwise_fma((v2f){w.z, w.w}, (v2f){x.z, x.w}, acc);
}
__device__ __forceinline__ float hsum(const v2f a) { return a.x + a.y; }

// Group formation of the persistent kernels, run by thread 0 of every workgroup: a group is
// whatever shares an XCD (HW_REG_XCC_ID), placement-independent. Returns 1 when all kPG * kPM
// workgroups registered, 32 per XCD; 0 (with PC_ERR set) on a registration timeout, a bad
// spread, or an error an earlier launch of the same call left in PC_ERR -- so a call whose
// first launch could not become co-resident drains its queued launches at once.
__device__ __forceinline__ int p_register(unsigned* ctl, int& group, int& slot) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    group = (int)(x & 7);
    slot = (int)atomicAdd(ctl + PC_REG + group, 1u);
    atomicAdd(ctl + PC_TOTAL, 1u);
    const unsigned t0 = p_now();
    while (ld_sc1_u(ctl + PC_TOTAL) < (unsigned)(kPG * kPM)) {
        if (ld_sc1_u(ctl + PC_ERR)) return 0;
        __builtin_amdgcn_s_sleep(1);
        if (p_now() - t0 > kSpinTicks) {
            atomicMax(ctl + PC_ERR, 1u);
            return 0;
        }
    }
    if (ld_sc1_u(ctl + PC_ERR)) return 0;
    for (int i = 0; i < kPG; ++i)
        if (ld_sc1_u(ctl + PC_REG + i) != (unsigned)kPM) {
            atomicMax(ctl + PC_ERR, 3u);
            return 0;
        }
    return 1;
}

// Host side, before every persistent launch: can the launch's kPG * kPM workgroups be
// co-resident on this device (occupancy query at the launch's dynamic LDS, x the CU count)?
// A launch that could not be fails here in microseconds (hipErrorCooperativeLaunchTooLarge,
// reported by the runtime as "cannot become co-resident") instead of spinning in p_register.
// The answer is cached per kernel variant (`cached`: 0 unknown, 1 yes, 2 no). Test hook:
// WRNN_DEBUG_PERSIST_FAIL=occupancy makes the check fail.
inline hipError_t persist_coresident(const void* fn, size_t lds, int* cached) {
    if (const char* e = std::getenv("WRNN_DEBUG_PERSIST_FAIL"))
        if (!std::strcmp(e, "occupancy")) return hipErrorCooperativeLaunchTooLarge;
    if (*cached == 0) {
        int dev = 0, cus = 0, nb = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, kPT, lds);
        if (e != hipSuccess) return e;
        *cached = nb * cus >= kPG * kPM ? 1 : 2;
    }
    return *cached == 1 ? hipSuccess : hipErrorCooperativeLaunchTooLarge;
}

// Host side: launch one persistent kernel instance K (kPG * kPM workgroups of kPT threads,
// `lds` bytes of dynamic LDS): its LDS attribute once, the co-residency check, the launch.
template <auto K, typename Args>
inline hipError_t persist_launch(size_t lds, const Args& a, hipStream_t s) {
    const void* fn = reinterpret_cast<const void*>(K);
    static bool attr = false;
    if (!attr) {
        if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); e != hipSuccess)
            return e;
        attr = true;
    }
    static int coresident = 0;
    if (hipError_t e = persist_coresident(fn, lds, &coresident); e != hipSuccess) return e;
    hipLaunchKernelGGL(K, dim3(kPG * kPM), dim3(kPT), lds, s, a);
    return hipGetLastError();
}

// Progress of a launch for the host's progress callback (fatchord_version.py:234-236 calls
// back at i % 100 == 0): after step t with t % 100 == 0, one lane publishes base + t + 1
// steps done to a host-mapped word (vector store, system scope); the host polls it while the
// launch runs. base = row batch * S.
__device__ __forceinline__ void p_progress(unsigned* prog, int base, int value, int t) {
    if (prog != nullptr && t % kProgressEvery == 0)
        __hip_atomic_store(prog, (unsigned)(base + value + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void p_progress(unsigned* prog, int base, int t) { p_progress(prog, base, t, t); }

// Abort request of the host (the progress callback returned non-zero): the host sets the
// host-mapped word kAbortWord words past the progress word. At its progress points (every 100
// steps, and only when a callback is registered) slot 0 of EVERY group reads it; on a request
// it sets PC_ERR = 4 and returns true, and its workgroup exits at its next failure check --
// the group's other workgroups then give up at their next spin check, so the launch (and,
// through PC_ERR at registration, every queued launch of the call) drains within ~100 steps.
__device__ __forceinline__ bool p_abort(unsigned* ctl, const unsigned* prog, int t) {
    if (prog == nullptr || t % kProgressEvery != 0) return false;
    if (__hip_atomic_load(prog + kAbortWord, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) return false;
    atomicMax(ctl + PC_ERR, 4u);
    return true;
}

// Teacher-forced logit gate (debug only): the logit l of (row, cls) at a step the host asked
// for goes to dbg.out[slot][row][cls] (wrnn_debug_logits); nothing when the capture is off.
// Only the DBG instances of the kernels record (launched when the capture is on), so the
// production instances carry no trace of it (registers are at the limit there).
template <bool DBG>
__device__ __forceinline__ void p_dbg_logit(const DbgLogits& d, int t, int row, int cls, int B,
                                            int n, float l) {
    if constexpr (!DBG) return;
    if (d.out == nullptr) return;
    // (per lane: the lanes of one wave can hold rows at different step offsets -- a time-sliced
    // wide launch)
    const int k = d.map[t];
    if (k >= 0) d.out[((size_t)k * B + row) * n + cls] = l;
}

__device__ __forceinline__ int p_frame(const RowInfo& ri, int t, int hop) {
    const int rel = ri.rel0 + t;
    return rel < ri.L ? ri.fbase + 1 + rel / hop : ri.fbase;
}

template <int CTRL>
__device__ __forceinline__ int pdpp_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
// (v, k) <- (v2, k2) when v2 is larger, or equal with a lower class. Bitwise, not `||` / `&&`:
// the short-circuit form compiled to exec-mask branches (~17 instructions per step on the
// candidate publish and sample paths); this is compares + two v_cndmask
__device__ __forceinline__ void amax_take(float& v, int& k, float v2, int k2) {
    const bool take = (v2 > v) | ((v2 == v) & (k2 < k));
    v = take ? v2 : v;
    k = take ? k2 : k;
}
template <int CTRL>
__device__ __forceinline__ void amax_dpp_step(float& v, int& k) {
    const float v2 = pdpp<CTRL>(v);
    const int k2 = pdpp_i<CTRL>(k);
    amax_take(v, k, v2, k2);
}
// argmax over the 16 lanes of a DPP row (value, class); ties -> lowest class; all lanes get it
__device__ __forceinline__ void row16_argmax(float& v, int& k) {
    amax_dpp_step<0xB1>(v, k);
    amax_dpp_step<0x4E>(v, k);
    amax_dpp_step<0x124>(v, k);
    amax_dpp_step<0x128>(v, k);
}

// RAW hop D carries its own sequence tag: each slot writes one 64-bit word per row (the
// candidate key below, tag in its low byte), so consumers poll the candidates themselves.
typedef unsigned u2v __attribute__((ext_vector_type(2)));
constexpr unsigned kTagSeqMask = (1u << 21) - 1;  // steps per call < 2^21 (host-checked)

// argmax over the 32 lanes of a half-wave (value, class); ties -> lowest class. DPP only:
// each 16-lane row reduces itself, then row_bcast:15 hands row 0's (row 2's) result to row 1
// (row 3). The half-wave's result is valid in its upper 16 lanes (lane & 31 >= 16).
__device__ __forceinline__ void half_argmax(float& v, int& k) {
    row16_argmax(v, k);
    const float v2 = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x142, 0xA, 0xF, false));
    const int k2 = __builtin_amdgcn_update_dpp(k, k, 0x142, 0xA, 0xF, false);
    amax_take(v, k, v2, k2);
}

// Buffer-resource access: a uniform (SGPR) base and a 32-bit per-lane byte offset, so no
// 64-bit per-lane addresses stay live across the step loop.
typedef __amdgpu_buffer_rsrc_t rsrc_t;
// cache policy of the polls: non-temporal (served by L2, bypasses the CU's L1); sc1 measured
// the same (6.661 vs 6.677 us per C2 step)
constexpr int kCpNT = 2;
__device__ __forceinline__ rsrc_t mk_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float bld(rsrc_t r, unsigned voff, unsigned soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
__device__ __forceinline__ float bld_nt(rsrc_t r, unsigned voff, unsigned soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, kCpNT));
}
__device__ __forceinline__ float4 bld4_nt(rsrc_t r, unsigned voff, unsigned soff) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, kCpNT));
}
__device__ __forceinline__ void bst(float v, rsrc_t r, unsigned voff, unsigned soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, voff, soff, 0);
}

typedef unsigned u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bst_tag(float v, unsigned tag, rsrc_t r, unsigned voff, unsigned soff) {
    __builtin_amdgcn_raw_buffer_store_b64((u2v){__float_as_uint(v), tag}, r, voff, soff, 0);
}
// Poll M 16-byte couples (two tagged pairs each) until every tag equals `want`, storing the
// values to LDS (dst[m], float2) on every pass; the last pass, the one that saw all tags, wins.
// False on an abort / timeout (error code set).
template <int M, bool ALL_FIRST = false>
__device__ __forceinline__ bool poll_couples(rsrc_t xr, const unsigned (&off)[M], unsigned so,
                                             unsigned want, float2* const (&dst)[M], unsigned* ctl) {
    // spin on the first couple only (a thread's couples all come from one producer slot), then
    // take the whole set and verify every tag; keeps the polling traffic in L2 small. Two
    // polls stay in flight (the next is issued before the previous is checked), so a landed
    // value is seen about half an L2 round trip sooner than with one poll at a time.
    const unsigned t0 = p_now();
    unsigned n = 0;
    if constexpr (ALL_FIRST) {
        // first pass: every couple in flight at once -- when the data is there already this is
        // one L2 round trip instead of two (measured per kernel: geneing 3.73 -> 3.57 us/step;
        // fatchord 6.53 -> 6.72 and runtimeracer 8.67 -> 8.83 slower, so geneing only)
        bool ok = true;
        u4v c[M];
#pragma unroll
        for (int m = 0; m < M; ++m) c[m] = __builtin_amdgcn_raw_buffer_load_b128(xr, off[m], so, kCpNT);
#pragma unroll
        for (int m = 0; m < M; ++m) {
            *dst[m] = make_float2(__uint_as_float(c[m].x), __uint_as_float(c[m].z));
            ok = ok && c[m].y == want && c[m].w == want;
        }
        if (__all(ok)) return true;
    }
    u4v c0 = __builtin_amdgcn_raw_buffer_load_b128(xr, off[0], so, kCpNT);
    while (true) {
        const u4v c1 = __builtin_amdgcn_raw_buffer_load_b128(xr, off[0], so, kCpNT);
        if (__all(c0.y == want && c0.w == want)) {
            bool ok = true;
            *dst[0] = make_float2(__uint_as_float(c0.x), __uint_as_float(c0.z));
#pragma unroll
            for (int m = 1; m < M; ++m) {
                const u4v c = __builtin_amdgcn_raw_buffer_load_b128(xr, off[m], so, kCpNT);
                *dst[m] = make_float2(__uint_as_float(c.x), __uint_as_float(c.z));
                ok = ok && c.y == want && c.w == want;
            }
            if (__all(ok)) return true;
        }
        c0 = c1;
        if ((++n & 63) == 0 && (ld_sc1_u(ctl + PC_ERR) || p_now() - t0 > kSpinTicks)) {
            if ((threadIdx.x & 63) == 0) atomicMax(ctl + PC_ERR, 2u);
            return false;
        }
    }
}

}  // namespace wrnn
