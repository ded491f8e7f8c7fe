// EXPERIMENT (not built): the wide-row kernel with one 512-register wave per SIMD (4 waves,
// K quarters, off-path products in the hop waits). Bit-exact on MI355X but 16.5 us/step vs
// 13.2 for the 8-wave kernel (profiles/r02/phase_wide4w.log): AGPR-resident weights are copied
// to VGPRs per MFMA and one wave per SIMD cannot overlap epilogues with matrix work.

// Persistent fatchord recurrence for WIDE row batches (the "persist-wide" launch kind):
// up to 16 fold rows per XCD group, 128 rows per launch, the matrix-vector products of every
// step on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32, the fp32 vector rate).
//
// Reference step body: vocoder/models/fatchord_version.py:192-236 (same restructuring as
// kernels_persist.hip: conditioning hoisted into per-frame / per-step precomputes, torch
// GRUCell arithmetic). What changes at 16 rows per group:
//  * Products as MFMA tiles. A workgroup (slot w of its XCD group) owns units / outputs
//    [16w, 16w + 16) of every layer and classes [16w, 16w + 16) of fc3: one 16-row M tile per
//    gate matrix; the group's rows are the 16 N columns. One 512-register wave per SIMD (4
//    waves): wave v takes the K quarter [128v, 128v + 128) (32 k-steps of 4); the 4 partial
//    tiles are summed in LDS in a fixed order (deterministic). Weights stay resident: 9 tiles
//    per wave in registers (W_ih2[:, :512] r/z/n, W_hh1 r/z/n, fc1, fc2, fc3), W_hh2 r/z/n in
//    LDS.
//  * GRU1 distributed, not redundant: each slot runs GRU1 for its own 16 units x rows and
//    publishes x1 / h1 (redundant GRU1 of all 512 units would cost 16x the cell work here).
//    Five in-group hops per step: E (x1, h1), A (x2, h2), B (y1), C (y2), D (fc3 candidates).
//  * Exchange: every published vector is laid out as 16-byte couples {v(u), tag, v(u+1), tag}
//    in MFMA B-operand order ([wave e][couple i][k-slot c][row n]), so a consumer wave reads its
//    B operand straight into registers with 16 fully coalesced 1-KiB loads per hop and checks
//    the step tags itself -- no LDS staging of activations, no flags. Producers store with
//    plain vector stores; consumers load non-temporal (L2-served): both ends of every hop are
//    on one XCD (HW_REG_XCC_ID grouping), so the XCD's L2 is the coherence point (DESIGN.md,
//    "Memory ordering").
//  * Off-path products (W_hh1 h1 -> gh1 for this step's GRU1, W_hh2 h2 -> gh2 for the next
//    step's GRU2) run in the hop waits ("slots"): their B operands are loaded right after the
//    previous critical products, the next hop's first couple is peeked, the off-path MFMAs are
//    issued, and only then is the hop polled. Slot A (hop A): W_hh1 h1 (3 tiles); slot B
//    (hop B): W_hh2 h2 r, z; slot C (hop C): W_hh2 h2 n.
// Every spin is bounded; on a timeout / error the kernel sets PC_ERR and every wave exits at
// its next barrier.
#include "wrnn_kernels.h"
#include "persist_common.h"

namespace wrnn {

typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int kWW = 4;            // waves per workgroup (one per SIMD)
constexpr int kWThr = 64 * kWW;   // threads per workgroup
constexpr int kWKS = 32;          // k-steps per wave (K quarter / 4)
constexpr int kWC = kWKS / 2;     // 16-byte couples per lane per hop

// ---- exchange area per group (floats) ---------------------------------------------------
constexpr int WV = kWW * kWC * 4 * 16 * 4;  // one vector buffer: [e 4][i 16][c 4][n 16] couples
enum WBuf : int { WB_X1 = 0, WB_H1, WB_X2, WB_H2, WB_Y1, WB_Y2, WB_N };
constexpr int WX_D = WB_N * WV;                    // candidates [n 16][slot 32] (value, tag|class)
constexpr int WX_GROUP = WX_D + 16 * 32 * 2 + 64;

// ---- LDS (floats) -------------------------------------------------------------------------
constexpr int WL_X1 = 0;                         // x1 of the slot's units [16 n][16 ul]
constexpr int WL_SX = WL_X1 + 256;               // sample per row [16]
constexpr int WL_CV = WL_SX + 16;                // hop-D partial argmax [4][16] value, class
constexpr int WL_CI = WL_CV + 64;
constexpr int WL_RI = WL_CI + 64;                // RowInfo of the group's rows (6 words each)
constexpr int WL_FAIL = WL_RI + 16 * 6;
constexpr int WL_REG = WL_FAIL + 4;              // group, slot, registration result (ints)
constexpr int WL_PS = 512;                       // 1-tile partials [4 v][16 n][16 o]
constexpr int WL_PA = WL_PS + kWW * 256;         // 3-tile partials [4 v][3][16 n][16 o]: W_ih2 x1
constexpr int WL_PE = WL_PA + kWW * 3 * 256;     //   W_hh2 h2 (gh2 of the next step)
constexpr int WL_PH = WL_PE + kWW * 3 * 256;     //   W_hh1 h1 (gh1)
constexpr int WL_HH2 = WL_PH + kWW * 3 * 256;    // W_hh2 r, z, n tiles: [3][4 v][8 q][64 l][4]
constexpr int WL_HH2_SZ = 3 * kWW * kWKS * 64;
constexpr int WL_TOTAL = WL_HH2 + WL_HH2_SZ;
static_assert(WL_REG + 4 <= WL_PS, "small LDS arrays overflow their 2 KiB");
static_assert(WL_TOTAL * 4 <= 160 * 1024, "LDS carve exceeds the CU's 160 KiB (no static LDS)");
static_assert(sizeof(RowInfo) == 24, "RowInfo is 6 words");

// register tiles of a wave: 0-2 W_ih2x r,z,n | 3-5 W_hh1 r,z,n | 6 fc1 | 7 fc2 | 8 fc3
constexpr int kWTiles = 9;
constexpr int kWQ = kWTiles * kWKS / 4;  // float4 weight registers per lane (72)

__device__ __forceinline__ v4f mfma4(float a, float b, v4f c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float f4c(const float4& q, int i) {
    return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
}
// B operand of k-step ks from the couples of a hop (couple i holds k-steps 2i, 2i + 1)
__device__ __forceinline__ float bop(const u4v (&cc)[kWC], int ks) {
    return __uint_as_float((ks & 1) ? cc[ks >> 1].z : cc[ks >> 1].x);
}

// LDS-only workgroup barrier: no wait on outstanding global loads (prefetches stay in flight)
__device__ __forceinline__ void wbar() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// This lane's couples of one hop buffer: byte offset of couple 0 = voff, couple i at
// voff + 1 KiB i. Lanes with valid == false (rows beyond the group's count) hold zeros.
//   w_issue  loads all couples (no wait: the caller overlaps them with other work)
//   w_check  waits for them, verifies the step tags and re-polls if any is stale
//   w_poll   polls couple 0 (starting from a couple 0 loaded earlier by w_peek) until its
//            tags match, then loads and verifies the rest
__device__ __forceinline__ void w_issue(rsrc_t xr, unsigned voff, unsigned so, unsigned want,
                                        bool valid, u4v (&cc)[kWC]) {
    unsigned vo = voff;
    asm volatile("" : "+v"(vo));  // (offsets recomputed per use: hoisted ones pin registers)
#pragma unroll
    for (int i = 0; i < kWC; ++i)
        cc[i] = valid ? __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024u * i, so, kCpNT)
                      : (u4v){0u, want, 0u, want};
}
__device__ __forceinline__ bool w_tags(const u4v (&cc)[kWC], unsigned want) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < kWC; ++i) ok = ok && cc[i].y == want && cc[i].w == want;
    return ok;
}
__device__ __forceinline__ u4v w_peek(rsrc_t xr, unsigned voff, unsigned so, unsigned want, bool valid) {
    return valid ? __builtin_amdgcn_raw_buffer_load_b128(xr, voff, so, kCpNT) : (u4v){0u, want, 0u, want};
}
__device__ __forceinline__ bool w_poll(rsrc_t xr, unsigned voff, unsigned so, unsigned want,
                                       bool valid, u4v (&cc)[kWC], unsigned* ctl, u4v first) {
    const unsigned t0 = p_now();
    unsigned nsp = 0;
    cc[0] = first;
    while (true) {
        if (__all(cc[0].y == want && cc[0].w == want)) {
            unsigned vo = voff;
            asm volatile("" : "+v"(vo));
#pragma unroll
            for (int i = 1; i < kWC; ++i)
                cc[i] = valid ? __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024u * i, so, kCpNT)
                              : (u4v){0u, want, 0u, want};
            if (__all(w_tags(cc, want))) return true;
        }
        if ((++nsp & 63) == 0 && (ld_sc1_u(ctl + PC_ERR) || p_now() - t0 > kSpinTicks)) {
            if ((threadIdx.x & 63) == 0) atomicMax(ctl + PC_ERR, 2u);
            return false;
        }
        cc[0] = w_peek(xr, voff, so, want, valid);
    }
}
__device__ __forceinline__ bool w_check(rsrc_t xr, unsigned voff, unsigned so, unsigned want,
                                        bool valid, u4v (&cc)[kWC], unsigned* ctl) {
    if (__all(w_tags(cc, want))) return true;
    return w_poll(xr, voff, so, want, valid, cc, ctl, w_peek(xr, voff, so, want, valid));
}

__global__ __launch_bounds__(kWThr, 1) void k_persist_wide(PersistArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    int* sreg = reinterpret_cast<int*>(lds + WL_REG);
    const int tid = threadIdx.x;
    if (tid == 0) {
        int gg, ss;
        sreg[2] = p_register(a.ctl, gg, ss);
        sreg[0] = gg;
        sreg[1] = ss;
    }
    __syncthreads();
    if (!sreg[2]) return;
    const int g = __builtin_amdgcn_readfirstlane(sreg[0]);
    const int w = __builtin_amdgcn_readfirstlane(sreg[1]);
    const int v = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave: K quarter [128v, 128v + 128)
    const int l = tid & 63;
    const int R = a.nr;                  // rows of this group (<= 16)
    const int g0 = a.rb + g;             // group row r = fold row g0 + 8 r
    const int bn = l & 15;               // B-operand lane: row bn, k-slot l >> 4
    const bool bvalid = bn < R;
    // epilogue cell of threads 0..16R-1: row cn, unit / class 16 w + cul
    const int cn = tid >> 4, cul = tid & 15;
    const bool cell = tid < 16 * R;
    const int cu = 16 * w + cul;
    const int crow = g0 + kPG * (cell ? cn : 0);
    const rsrc_t xr = mk_rsrc(a.xbuf + (size_t)g * WX_GROUP);
    const bool trace = a.phases != nullptr;
    uint32_t* ph = trace ? a.phases + (size_t)(g * kPM + w) * kPPhases : nullptr;
#define WSTAMP(i) \
    if (trace && t == a.phase_t && tid == 0) ph[(i)] = p_now();

    // ---- weights ------------------------------------------------------------------------
    float4 wq[kWQ];  // tile T, k-step ks: wq[8T + ks / 4] component ks % 4
    {
        const float4* src = a.wwide + ((size_t)(w * kWW + v) * kWQ) * 64 + l;
#pragma unroll
        for (int q = 0; q < kWQ; ++q) wq[q] = src[(size_t)q * 64];
        const float4* hs = a.wwide_lds + (size_t)w * (WL_HH2_SZ / 4);
        float4* hd = reinterpret_cast<float4*>(lds + WL_HH2);
        for (int i = tid; i < WL_HH2_SZ / 4; i += kWThr) hd[i] = hs[i];
    }
#define WR(T, ks) f4c(wq[8 * (T) + (ks) / 4], (ks) % 4)
    const float4* hh2 = reinterpret_cast<const float4*>(lds + WL_HH2);
    // ---- state and per-cell constants --------------------------------------------------
    float h1r = 0.f, h2r = 0.f, vj[3] = {0.f, 0.f, 0.f}, w0u = 0.f, bh1[3] = {0.f, 0.f, 0.f},
          bh2[3] = {0.f, 0.f, 0.f}, g2i[3] = {0.f, 0.f, 0.f}, bf3 = 0.f;
    if (cell) {
        h1r = a.st_h1[(size_t)crow * kPH + cu];
        h2r = a.st_h2[(size_t)crow * kPH + cu];
        lds[WL_X1 + cn * 16 + cul] = a.st_x1[(size_t)crow * kPH + cu];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            g2i[j] = a.st_gh2[(size_t)crow * 3 * kPH + j * kPH + cu];  // gh2 of step t0
            vj[j] = a.v[j * kPH + cu];
            bh1[j] = a.b_hh1[j * kPH + cu];
            bh2[j] = a.b_hh2[j * kPH + cu];
        }
        w0u = a.w0[cu];
        bf3 = cu < a.n_classes ? a.b_fc3[cu] : 0.f;
    }
    if (tid < R) reinterpret_cast<RowInfo*>(lds + WL_RI)[tid] = a.rows[g0 + kPG * tid];
    if (tid == 0) lds[WL_FAIL] = 0.f;
    // byte offsets: this lane's couple 0 in a hop buffer (consumer); the cell pair's couple
    // (producer: even units publish the pair {u, u + 1})
    const unsigned o_cons = (unsigned)((v * kWC * 64 + l) * 16);
    const unsigned o_prod =
        (unsigned)((((((w >> 3) * kWC + (w & 1) * 8 + (cul >> 1)) * 4 + ((w & 7) >> 1)) * 16) + cn) * 16);
    auto pub = [&](int hb, float val, unsigned tag) {
        const float nb = pdpp<0xB1>(val);  // unit u ^ 1 of the same row (quad_perm xor 1)
        if (cell && (cul & 1) == 0)
            __builtin_amdgcn_raw_buffer_store_b128((u4v){__float_as_uint(val), tag, __float_as_uint(nb), tag},
                                                   xr, o_prod, (unsigned)(hb * WV) * 4u, 0);
    };
    const rsrc_t fcr = mk_rsrc(a.fcond);
    // per-step operands of the cell, loaded right after the hop E poll:
    //   pc[0..2] GRU2 cond (W_ih2[:, 512:] a2 + b_ih2), pc[3] fc1 cond, pc[4] fc2 cond (frame t)
    //   pg       Gumbel noise of (row, class cu) at step t
    //   pp       P1(t + 1) of (row, unit cu): r, z, n of W_ih1 I(c) + b_ih1, then cI
    float pc[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, pg = 0.f;
    float4 pp = make_float4(0.f, 0.f, 0.f, 0.f);
    auto prefetch = [&](int t) {
        if (!cell) return;
        const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + WL_RI)[cn];
        const unsigned fo = (unsigned)(p_frame(ri, t, a.hop) * a.cond_width) * 4u;
        int uu = cu;
        asm volatile("" : "+v"(uu));  // (recomputed per step: hoisted offsets cost registers)
        pc[0] = bld(fcr, fo + (unsigned)(a.oG2 + uu) * 4u, 0);
        pc[1] = bld(fcr, fo + (unsigned)(a.oG2 + kPH + uu) * 4u, 0);
        pc[2] = bld(fcr, fo + (unsigned)(a.oG2 + 2 * kPH + uu) * 4u, 0);
        pc[3] = bld(fcr, fo + (unsigned)(a.oF1 + uu) * 4u, 0);
        pc[4] = bld(fcr, fo + (unsigned)(a.oF2 + uu) * 4u, 0);
        pg = bld(mk_rsrc(a.gumbel + ((size_t)t * a.B + crow) * a.n_classes), (unsigned)uu * 4u, 0);
        const int tn = t + 1 < a.S ? t + 1 : a.S - 1;
        pp = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                            mk_rsrc(a.P1 + ((size_t)tn * a.B + crow) * 4 * kPH),
                                            (unsigned)uu * 16u, 0, 0));
    };
    // partial tile of this wave: [v][tile][n][o] with o = 4 (l >> 4) + register
    const int pw = (v * 3 * 16 + bn) * 16 + 4 * (l >> 4);
    auto put3 = [&](int base, const v4f (&acc)[3]) {
#pragma unroll
        for (int j = 0; j < 3; ++j) *reinterpret_cast<v4f*>(lds + base + pw + j * 256) = acc[j];
    };
    // cell sums of the 4 partial tiles (fixed order)
    auto sum4 = [&](int base) {
        float s = 0.f;
#pragma unroll
        for (int vv = 0; vv < kWW; ++vv) s += lds[base + vv * 3 * 256 + cn * 16 + cul];
        return s;
    };
    auto sum4s = [&]() {  // 1-tile partials
        float s = 0.f;
#pragma unroll
        for (int vv = 0; vv < kWW; ++vv) s += lds[WL_PS + (vv * 16 + cn) * 16 + cul];
        return s;
    };
    auto put1 = [&](v4f acc) {
        *reinterpret_cast<v4f*>(lds + WL_PS + (v * 16 + bn) * 16 + 4 * (l >> 4)) = acc;
    };
    // single-tile product of register tile T: two accumulation chains (even / odd k-steps)
    auto mm1 = [&](int T, const u4v (&cc)[kWC]) {
        v4f e0 = {0.f, 0.f, 0.f, 0.f}, e1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < kWKS; ks += 2) {
            e0 = mfma4(WR(T, ks), bop(cc, ks), e0);
            e1 = mfma4(WR(T, ks + 1), bop(cc, ks + 1), e1);
        }
        return e0 + e1;
    };
    // W_hh2 product of LDS tile j (0 r, 1 z, 2 n)
    auto mm_hh2 = [&](int j, const u4v (&cc)[kWC]) {
        v4f e0 = {0.f, 0.f, 0.f, 0.f}, e1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < kWKS / 4; ++q) {
            __builtin_amdgcn_sched_barrier(0);  // one k-quad of LDS weights live at a time
            const float4 aw = hh2[((j * kWW + v) * (kWKS / 4) + q) * 64 + l];
            e0 = mfma4(aw.x, bop(cc, 4 * q), e0);
            e1 = mfma4(aw.y, bop(cc, 4 * q + 1), e1);
            e0 = mfma4(aw.z, bop(cc, 4 * q + 2), e0);
            e1 = mfma4(aw.w, bop(cc, 4 * q + 3), e1);
        }
        return e0 + e1;
    };
    __syncthreads();
    // initial hop E: x1, h1 of step t0 (k_persist_init) with tag t0 + 1
    pub(WB_X1, cell ? lds[WL_X1 + cn * 16 + cul] : 0.f, (unsigned)a.t0 + 1u);
    pub(WB_H1, h1r, (unsigned)a.t0 + 1u);
    const unsigned so_x1 = (unsigned)(WB_X1 * WV) * 4u, so_h1 = (unsigned)(WB_H1 * WV) * 4u;
    const unsigned so_x2 = (unsigned)(WB_X2 * WV) * 4u, so_h2 = (unsigned)(WB_H2 * WV) * 4u;
    const unsigned so_y1 = (unsigned)(WB_Y1 * WV) * 4u, so_y2 = (unsigned)(WB_Y2 * WV) * 4u;
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[0] = p_now();
    for (int t = a.t0; t < a.t1; ++t) {
        const unsigned seq = (unsigned)t + 1u;
        u4v cc[kWC];
        bool fail = false;
        WSTAMP(0);
        // ================= hop E -> stage A: W_ih2[:, :512] x1 (critical) ==================
        fail |= !w_poll(xr, o_cons, so_x1, seq, bvalid, cc, a.ctl, w_peek(xr, o_cons, so_x1, seq, bvalid));
        prefetch(t);
        WSTAMP(1);
        {
            v4f acc[3] = {(v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ks = 0; ks < kWKS; ++ks) {
                const float b = bop(cc, ks);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[j] = mfma4(WR(j, ks), b, acc[j]);
            }
            put3(WL_PA, acc);
        }
        w_issue(xr, o_cons, so_h1, seq, bvalid, cc);  // slot A operand (h1 of this step)
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(2);
        if (lds[WL_FAIL] != 0.f) return;
        // ================= GRU2 epilogue -> publish x2, h2 ==================================
        {
            float x2 = 0.f;
            if (cell) {
                float gi[3], gh[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    gi[j] = p_add(sum4(WL_PA + j * 256), pc[j]);
                    gh[j] = t == a.t0 ? g2i[j] : p_add(sum4(WL_PE + j * 256), bh2[j]);
                }
                h2r = p_gru(gi[0], gi[1], gi[2], gh[0], gh[1], gh[2], h2r);
                x2 = p_add(lds[WL_X1 + cn * 16 + cul], h2r);
            }
            pub(WB_X2, x2, seq);
            pub(WB_H2, h2r, seq);
        }
        WSTAMP(3);
        // ================= slot A: W_hh1 h1 -> gh1 partials | hop A -> stage B (fc1 x2) =====
        {
            const u4v pk = w_peek(xr, o_cons, so_x2, seq, bvalid);
            fail |= !w_check(xr, o_cons, so_h1, seq, bvalid, cc, a.ctl);
            v4f acc[3] = {(v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ks = 0; ks < kWKS; ++ks) {
                const float b = bop(cc, ks);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[j] = mfma4(WR(3 + j, ks), b, acc[j]);
            }
            put3(WL_PH, acc);
            fail |= !w_poll(xr, o_cons, so_x2, seq, bvalid, cc, a.ctl, pk);
        }
        WSTAMP(4);
        put1(mm1(6, cc));
        w_issue(xr, o_cons, so_h2, seq, bvalid, cc);  // slot B operand (h2 of this step)
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(5);
        if (lds[WL_FAIL] != 0.f) return;
        // fc1 epilogue: y1 = relu(fc1 x2 + fc1[:, 512:] a3 + b) -> publish
        {
            float y = 0.f;
            if (cell) {
                y = p_add(sum4s(), pc[3]);
                y = y > 0.f ? y : 0.f;
            }
            pub(WB_Y1, y, seq);
        }
        // ================= slot B: W_hh2 h2 (r, z) | hop B -> stage C (fc2 y1) ==============
        {
            const u4v pk = w_peek(xr, o_cons, so_y1, seq, bvalid);
            fail |= !w_check(xr, o_cons, so_h2, seq, bvalid, cc, a.ctl);
            const v4f er = mm_hh2(0, cc);
            *reinterpret_cast<v4f*>(lds + WL_PE + pw) = er;
            const v4f ez = mm_hh2(1, cc);
            *reinterpret_cast<v4f*>(lds + WL_PE + pw + 256) = ez;
            fail |= !w_poll(xr, o_cons, so_y1, seq, bvalid, cc, a.ctl, pk);
        }
        WSTAMP(6);
        put1(mm1(7, cc));
        w_issue(xr, o_cons, so_h2, seq, bvalid, cc);  // slot C operand (h2 again)
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(7);
        if (lds[WL_FAIL] != 0.f) return;
        {  // fc2 epilogue: y2 = relu(fc2 y1 + fc2[:, 512:] a4 + b) -> publish
            float y = 0.f;
            if (cell) {
                y = p_add(sum4s(), pc[4]);
                y = y > 0.f ? y : 0.f;
            }
            pub(WB_Y2, y, seq);
        }
        // ================= slot C: W_hh2 h2 (n) | hop C -> stage D (fc3 y2) =================
        {
            const u4v pk = w_peek(xr, o_cons, so_y2, seq, bvalid);
            fail |= !w_check(xr, o_cons, so_h2, seq, bvalid, cc, a.ctl);
            const v4f en = mm_hh2(2, cc);
            *reinterpret_cast<v4f*>(lds + WL_PE + pw + 512) = en;
            fail |= !w_poll(xr, o_cons, so_y2, seq, bvalid, cc, a.ctl, pk);
        }
        WSTAMP(8);
        put1(mm1(8, cc));
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(9);
        if (lds[WL_FAIL] != 0.f) return;
        // fc3 epilogue: candidate argmax_k (l_k + g_k) over the slot's 16 classes per row
        // (row cn = one DPP row of 16 lanes), published tagged by lane cul == 0
        const unsigned tag_hi = (seq & kTagSeqMask) << 11;
        {
            float val = -INFINITY;
            int cls = cu;
            if (cell && cu < a.n_classes) val = p_add(p_add(sum4s(), bf3), pg);
            row16_argmax(val, cls);
            if (cell && cul == 0)
                __builtin_amdgcn_raw_buffer_store_b64((u2v){__float_as_uint(val), tag_hi | (unsigned)cls}, xr,
                                                      (unsigned)((cn * 32 + w) * 2) * 4u, WX_D * 4, 0);
        }
        // ================= hop D: sample of step t (wave 0, every workgroup) ===============
        if (v == 0) {
            const int n = l & 15, gq = l >> 4;  // row n, slots 8 gq .. 8 gq + 7
            const bool valid = n < R;
            const unsigned off = (unsigned)((n * 32 + 8 * gq) * 2) * 4u;
            const unsigned want = seq & kTagSeqMask;
            u4v q[4] = {(u4v){0u, want << 11, 0u, want << 11}, (u4v){0u, want << 11, 0u, want << 11},
                        (u4v){0u, want << 11, 0u, want << 11}, (u4v){0u, want << 11, 0u, want << 11}};
            const unsigned t0s = p_now();
            unsigned nsp = 0;
            while (true) {
                bool ok = true;
                if (valid) {
                    unsigned vo = off;
                    asm volatile("" : "+v"(vo));
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        q[k] = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, WX_D * 4 + 16u * k, kCpNT);
#pragma unroll
                    for (int k = 0; k < 4; ++k) ok = ok && (q[k].y >> 11) == want && (q[k].w >> 11) == want;
                }
                if (__all(ok)) break;
                if ((++nsp & 63) == 0 && (ld_sc1_u(a.ctl + PC_ERR) || p_now() - t0s > kSpinTicks)) {
                    if (l == 0) atomicMax(a.ctl + PC_ERR, 2u);
                    fail = true;
                    break;
                }
            }
            float bv = -INFINITY;
            int bi = 0x7fffffff;
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // slots in ascending order; ties -> lowest class
                const float v0 = __uint_as_float(q[k].x), v1 = __uint_as_float(q[k].z);
                const int k0 = (int)(q[k].y & 0x7ffu), k1 = (int)(q[k].w & 0x7ffu);
                if (v0 > bv || (v0 == bv && k0 < bi)) { bv = v0; bi = k0; }
                if (v1 > bv || (v1 == bv && k1 < bi)) { bv = v1; bi = k1; }
            }
            lds[WL_CV + gq * 16 + n] = bv;
            lds[WL_CI + gq * 16 + n] = __int_as_float(bi);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (gq == 0 && valid) {
#pragma unroll
                for (int k = 1; k < 4; ++k) {
                    const float v2 = lds[WL_CV + k * 16 + n];
                    const int k2 = __float_as_int(lds[WL_CI + k * 16 + n]);
                    if (v2 > bv || (v2 == bv && k2 < bi)) { bv = v2; bi = k2; }
                }
                float xv;
                {
#pragma clang fp contract(off)
                    xv = (2.0f * (float)bi) / (float)(a.n_classes - 1) - 1.0f;
                }
                lds[WL_SX + n] = xv;
                if (w == 0) {
                    int nn = n;
                    asm volatile("" : "+v"(nn));
                    const unsigned ro = (unsigned)((g0 + kPG * nn) * a.ld);
                    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bi, mk_rsrc(a.labels), ro * 2u,
                                                          (unsigned)t * 2u, 0);
                    bst(xv, mk_rsrc(a.samples), ro * 4u, (unsigned)t * 4u);
                }
            }
        }
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(10);
        if (lds[WL_FAIL] != 0.f) return;
        // ================= GRU1 of step t + 1 for the slot's units -> publish x1, h1 ========
        //   gi = W_ih1 (cI + w0 x) + b_ih1 = P1 + v x ; x1 = (cI + w0 x) + h1
        // (at the last step it runs on clamped inputs and nobody reads the result)
        {
            float x1 = 0.f;
            if (cell) {
                const float x = lds[WL_SX + cn];
                float gh[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) gh[j] = p_add(sum4(WL_PH + j * 256), bh1[j]);
                h1r = p_gru(fmaf(vj[0], x, pp.x), fmaf(vj[1], x, pp.y), fmaf(vj[2], x, pp.z), gh[0], gh[1],
                            gh[2], h1r);
                x1 = p_add(fmaf(w0u, x, pp.w), h1r);
                lds[WL_X1 + cn * 16 + cul] = x1;
            }
            pub(WB_X1, x1, seq + 1u);
            pub(WB_H1, h1r, seq + 1u);
        }
        if (g == 0 && w == 0 && tid == 0) p_progress(a.progress, a.prog_base, t);
        WSTAMP(11);
    }
#undef WSTAMP
#undef WR
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[1] = p_now();
}

size_t persist_wide_lds_bytes() { return (size_t)WL_TOTAL * sizeof(float); }
size_t persist_wide_xbuf_floats() { return (size_t)kPG * WX_GROUP; }
size_t persist_wide_wreg_floats() { return (size_t)kPM * kWW * kWQ * 64 * 4; }
size_t persist_wide_wlds_floats() { return (size_t)kPM * WL_HH2_SZ; }
int persist_wide_waves() { return kWW; }

int persist_wide_scratch() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_persist_wide) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}

hipError_t launch_persist_wide(const PersistArgs& a, hipStream_t s) {
    if (a.rb < 0 || a.nr < 1 || a.nr > kPWideRows || a.rb + kPG * a.nr > a.B || a.n_classes > kPM * 16 ||
        a.mode != 0 || a.wwide == nullptr)
        return hipErrorInvalidValue;
    static bool attr = false;
    const size_t lds = persist_wide_lds_bytes();
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)k_persist_wide,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL(k_persist_wide, dim3(kPG * kPM), dim3(kWThr), lds, s, a);
    return hipGetLastError();
}

}  // namespace wrnn
