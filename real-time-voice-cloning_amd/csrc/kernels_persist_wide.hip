// Persistent fatchord recurrence for WIDE row batches (the "persist-wide" launch kind):
// up to 16 fold rows per XCD group, 128 rows per launch, the matrix-vector products of every
// step on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32, the fp32 vector rate).
//
// Reference step body: vocoder/models/fatchord_version.py:192-236 (same restructuring as
// kernels_persist.hip: conditioning hoisted into per-frame / per-step precomputes, torch
// GRUCell arithmetic). What changes at 16 rows per group:
//  * Products as MFMA tiles. A workgroup (slot w of its XCD group) owns units / outputs
//    [16w, 16w + 16) of every layer and classes [16w, 16w + 16) of fc3: one 16-row M tile per
//    gate matrix. The group's rows are the 16 N columns. K = 512 is split over the 8 waves
//    (wave v: units [64v, 64v + 64), 16 k-steps of 4); the 8 partial tiles are summed in LDS in
//    a fixed order (deterministic). Weights stay resident: 9 tiles per wave in registers
//    (W_ih2[:, :512] r/z/n, W_hh1 r/z/n, fc1, fc2, fc3), W_hh2 r/z/n in LDS.
//  * GRU1 distributed, not redundant: each slot runs GRU1 for its own 16 units x rows and
//    publishes x1 / h1 (redundant GRU1 of all 512 units would cost 16x the cell work here).
//    Five in-group hops per step: E (x1, h1), A (x2, h2), B (y1), C (y2), D (fc3 candidates).
//  * Exchange: every published vector is laid out as 16-byte packets of 4 floats in MFMA
//    B-operand order, two slots by step parity, so a consumer wave reads its B operand straight
//    into registers with 4 fully coalesced 1-KiB loads per hop. Untagged: the slot a producer
//    will write next holds a sentinel (see w_poll for why that is race-free), so a hop moves
//    4 B per value (a tagged pair moved 8) -- no LDS staging of activations, no flags.
//    Producers store with plain vector stores; consumers load non-temporal (L2-served): both
//    ends of every hop are on one XCD (HW_REG_XCC_ID grouping), so the XCD's L2 is the
//    coherence point ("Memory ordering").
//  * Off-path products (W_hh1 h1 -> gh1, W_hh2 h2 -> gh2 of the next step) run in the waits of
//    hops A and B; waves 4-7 (no epilogue cells) start them while waves 0-3 run the epilogues.
// Every spin is bounded; on a timeout / error the kernel sets PC_ERR and every wave exits at
// its next barrier.
#include "wrnn_kernels.h"
#include "persist_common.h"
#include "philox.h"
#include "wide_layout.h"

#include <vector>

namespace wrnn {

typedef float v4f __attribute__((ext_vector_type(4)));

// ---- exchange area per group (floats) ---------------------------------------------------
// One published vector (x1, h1, x2, h2, y1, y2) per step: two slots (step parity), each
// [e 8][p 4][lane 64] packets of 4 floats in MFMA B-operand order -- packet p of consumer lane
// l = 16 c + n of wave e holds row n, units 64 e + 16 c + 4 p + q (q = 0..3), i.e. the B operands
// of k-steps 4p..4p+3 (k-step ks of k-slot c is unit 64 e + 16 c + ks: the weight images' order,
// runtime.hip pack_persist_wide) -- then room for 1024 more floats. Untagged: a slot not yet written for
// the step holds the sentinel kSent (see pub / w_poll).
// (wide_layout.h: the formulas, shared with the host-side check wide_layout_check)
using wide::WS_MAIN;
using wide::WSLOT;
using wide::WV;
using wide::WX_D;
using wide::WX_GROUP;
constexpr unsigned kSent = 0x7fbadbadu;  // a signalling NaN: no arithmetic result is ever this
enum WBuf : int { WB_X1 = 0, WB_H1, WB_X2, WB_H2, WB_Y1, WB_Y2, WB_N };
static_assert(WB_N == wide::kBufs, "one slot pair per published vector");
// ---- LDS (floats) -------------------------------------------------------------------------
// Everything read per step sits in the first 64 KiB so every ds_read / ds_write offset fits
// the instruction's 16-bit immediate (beyond it each access would pin an address register).
constexpr int WL_RI = 0;                         // RowInfo of the group's rows (6 words each)
constexpr int WL_VM = WL_RI + 6 * kPWideRows;     // (physical row, step offset) of each row slot
constexpr int WL_FAIL = WL_VM + 2 * kPWideRows;
constexpr int WL_REG = WL_FAIL + 4;              // group, slot, registration result (ints)
constexpr int WL_BIAS = WL_REG + 4;              // b_hh1 [3][16], b_hh2 [3][16], b_fc3 [16 (+16)] of the slot
constexpr int WL_P1R = 512;                      // P1 ring: float4 [16 n][16 j] (one slot, p1_make)
constexpr int WL_GR = WL_P1R + 16 * 16 * 4;      // noise ring: [16 n][16 (C10: 32)] (one slot, noise_make)
constexpr int WL_PS = 2048;                      // 1-tile partials [8 v][16 n][16 o]
constexpr int WL_PA = WL_PS + 8 * 256;           // 3-tile partials [8 v][3][16 n][16 o]
constexpr int WL_PH = WL_PA + 8 * 3 * 256;       // W_hh1 h1 partials (same layout)
constexpr int WL_HH2 = WL_PH + 8 * 3 * 256;      // W_hh2 r, z, n tiles: [3][8 v][4 q][64 l][4]
constexpr int WL_HH2_SZ = 3 * 8 * 16 * 64;
constexpr int WL_TOTAL = WL_HH2 + WL_HH2_SZ;
static_assert(WL_BIAS + 128 <= WL_P1R && WL_GR + 16 * 32 <= WL_PS, "small LDS arrays overflow their region");
static_assert(WL_HH2 * 4 <= 65536, "per-step LDS arrays must fit the 16-bit ds offset");
static_assert(WL_TOTAL * 4 <= 160 * 1024, "LDS carve exceeds the CU's 160 KiB (no static LDS)");
static_assert(sizeof(RowInfo) == 24, "RowInfo is 6 words");

// register tiles of a wave: 0-2 W_ih2x r,z,n | 3-5 W_hh1 r,z,n | 6 fc1 | 7 fc2 | 8 fc3
constexpr int kWTiles = 9;

__device__ __forceinline__ v4f mfma4(float a, float b, v4f c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float f4c(const float4& q, int i) {
    return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
}
// B operand of k-step ks from the 4 packets of a hop (packet p holds k-steps 4p .. 4p + 3)
__device__ __forceinline__ float bop(const u4v (&cc)[4], int ks) {
    const u4v& q = cc[ks >> 2];
    return __uint_as_float((ks & 3) == 0 ? q.x : (ks & 3) == 1 ? q.y : (ks & 3) == 2 ? q.z : q.w);
}
// Partial tiles: element (row n, column o) of a [16][16] tile sits at n * 16 + wsw(n, o), the
// 16-byte column slots XOR-swizzled by row: an MFMA lane's 16-byte store (row bn, columns
// 4c .. 4c + 3) and the epilogue's row reads are then both conflict-free (a ds_write_b128 is
// served 8 contiguous lanes at a time on 32 banks: unswizzled, rows 64 B apart put 8 rows on 2
// slots -- 4-way, 24 extra LDS cycles per store, ~2300 per CU and step; SQ_LDS_BANK_CONFLICT,
// profiles/r03/pmc/c4_sq)
__device__ __forceinline__ int wsw(int n, int o) { return ((((o >> 2) ^ (n >> 1)) & 3) << 2) | (o & 3); }

__device__ __forceinline__ bool p_ready(const u4v& q) {
    // bitwise: the short-circuit form compiled to a branch and a wait per packet
    return (q.x != kSent) & (q.y != kSent) & (q.z != kSent) & (q.w != kSent);
}

// LDS-only workgroup barrier: no wait on outstanding global loads (prefetches stay in flight)
__device__ __forceinline__ void wbar() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Poll this lane's 4 packets of one hop buffer slot (byte offset of packet 0: voff; packet p at
// voff + 1 KiB p; so: the buffer and slot) until no value is the sentinel, all 4 in flight on
// every pass. Lanes with valid == false (rows beyond the group's count) contribute zeros.
// Why a sentinel is enough (no step tags): a producer writes step s into slot s & 1 and the
// sentinel into slot (s + 1) & 1 (pub). Its next poll waits for every older vector memory
// operation of the wave (vmcnt counts stores on gfx9), so that reset is in L2 before it
// publishes anything later; a consumer polls slot (s + 1) & 1 for step s + 1 only after it has
// read such a later publication, so it sees the reset or the new value, never step s - 1. And
// slot s & 1 is rewritten (step s + 2) only after every consumer has published past its reads
// of step s.
// The 4 packet loads of a poll round. Unconditional: a lane without an operand loads from an
// out-of-range offset, which reads 0 ("ready"), so every path carries the same loads and the
// compiler's waits stay counted (a branch around them made the waits after it conservative).
// w_issue alone: the first round issued early, for an off-path operand published long before
// its use, checked later by w_poll with pre = true.
__device__ __forceinline__ void w_issue(rsrc_t xr, unsigned voff, unsigned so, bool valid, u4v (&cc)[4]) {
    unsigned vo = valid ? voff : wide::kNoOffset;
    asm volatile("" : "+v"(vo));
#pragma unroll
    for (int i = 0; i < 4; ++i) cc[i] = __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024u * i, so, kCpNT);
}
// Packet i of a poll round alone (see w_issue): issued into a packet register an off-path
// product has finished reading, so a critical hop's first round needs no extra registers.
__device__ __forceinline__ void w_issue1(rsrc_t xr, unsigned voff, unsigned so, bool valid, u4v& c, int i) {
    unsigned vo = valid ? voff : wide::kNoOffset;
    asm volatile("" : "+v"(vo));
    c = __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024u * i, so, kCpNT);
}
// On a timeout the first poller records its site in PC_WHERE (`where`: site << 28 | slot << 22;
// the wave is added here), whether its packets were missing (PC_WHERE + 1) and the step
// (PC_WHERE + 2, all 32 bits), for the error message.
__device__ __forceinline__ bool w_poll(rsrc_t xr, unsigned voff, unsigned so, bool valid, u4v (&cc)[4],
                                       unsigned* ctl, unsigned where, unsigned step, bool pre = false) {
    const unsigned t0 = p_now();
    unsigned nsp = 0;
    if (!pre) w_issue(xr, voff, so, valid, cc);
    {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < 4; ++i) ok &= p_ready(cc[i]);
        if (__all(ok)) return true;
    }
    while (true) {
        // every packet reloaded per spin: a lane's 4 packets come from one producer slot's one
        // store instruction, so when packet 0 lands the others have too and no second L2 round
        // trip follows (round 3 A/B: 11.33 against 11.48 us per step spinning on packet 0,
        // profiles/r03/ab_spin/)
        w_issue(xr, voff, so, valid, cc);
        {
            bool ok = true;
#pragma unroll
            for (int i = 0; i < 4; ++i) ok &= p_ready(cc[i]);
            if (__all(ok)) return true;
        }
        if ((++nsp & 63) == 0 && (ld_sc1_u(ctl + PC_ERR) || p_now() - t0 > kSpinTicks)) {
            if (!ld_sc1_u(ctl + PC_ERR)) {  // the first to time out records where
                bool mok = true;
#pragma unroll
                for (int i = 0; i < 4; ++i) mok &= p_ready(cc[i]);
                const bool mbad = !__all(mok);
                // (the wave index read back as a scalar: a per-lane form was precomputed per site
                // before the step loop and held VGPRs)
                const unsigned wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
                if ((threadIdx.x & 63) == 0 && atomicCAS(ctl + PC_WHERE, 0u, where | (wv << 19)) == 0u) {
                    ctl[PC_WHERE + 1] = mbad ? 1u : 0u;
                    ctl[PC_WHERE + 2] = step;
                }
            }
            if ((threadIdx.x & 63) == 0) atomicMax(ctl + PC_ERR, 2u);
            return false;
        }
    }
}

// DBG: the instance that records logits for the teacher-forced gate (wrnn_set_debug_steps)
// ROT: a time-sliced launch (PersistArgs::vmap): row slot r of group g is the
//      virtual row v = g + 8 r, which a.vmap maps to (physical row, step offset); the launch runs
//      steps [0, t1) of its rows (their steps off .. off + t1 - 1) and saves their state at the end
// C10: up to 1024 classes (fatchord's 10-bit default): slot w also owns classes 512 + 16 w ..
//      512 + 16 w + 15, a second fc3 tile whose A operands (a.wfc3b, 1 MiB per group image,
//      L2-resident) are loaded every step right after the hop-C poll and consumed after the
//      first tile's MFMAs -- the registers hold the other nine tiles; its partials go to PH after
//      one more barrier (the gh1 / gh2 partial sums are read in the hop-C wait instead of hop D,
//      so PH is free by then)
template <bool ROT, bool C10, bool DBG>
__global__ __launch_bounds__(kPT, 1) void k_persist_wide(PersistArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];  // the whole 160 KiB
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
    const int v = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave: K-eighth [64v, 64v + 64)
    const int l = tid & 63;
    const int R = a.nr;                  // rows of this group (<= 16)
    const int g0 = a.rb + g;             // group row r = fold row g0 + 8 r
    const int bn = l & 15;               // B-operand lane: row bn, k-slot l >> 4
    const bool bvalid = bn < R;
    // epilogue cell of threads 0..16R-1: row cn, unit / class 16 w + cul
    const int cn = tid >> 4, cul = tid & 15;
    const bool cell = tid < 16 * R;
    const int cu = 16 * w + cul;
    // (physical) row of this lane's cell; a time-sliced launch maps the virtual row
    const int crow = ROT ? a.vmap[g0 + kPG * (cell ? cn : 0)].x : g0 + kPG * (cell ? cn : 0);
    // timeout site record (PC_WHERE): site << 28 | slot << 22 (| wave << 19, added by the poller);
    // the step goes to PC_WHERE + 2 whole
    // (recomputed per use from the scalar slot index: the hoisted constants held VGPRs)
    auto wh = [&](unsigned site) {
        unsigned ww = (unsigned)w;
        asm volatile("" : "+s"(ww));
        return site << 28 | ww << 22;
    };
    const rsrc_t xr = mk_rsrc(a.xbuf + (size_t)g * WX_GROUP);
    const bool trace = a.phases != nullptr;
    uint32_t* ph = trace ? a.phases + (size_t)(g * kPM + w) * kPPhases : nullptr;
#define WSTAMP(i)                                                             \
    if (trace && t == a.phase_t && (tid & 255) == 0) {                        \
        ph[(tid >> 8) * 12 + (i)] = p_now();                                  \
        if (tid == 0 && ((i) == 0 || (i) == 10))                              \
            ph[24 + ((i) == 10)] = (uint32_t)__builtin_amdgcn_s_memtime();    \
    }
    // extra stamps of wave 0 at [26, 32): inside the off-path windows
#define WXSTAMP(i) \
    if (trace && t == a.phase_t && tid == 0) ph[(i)] = p_now();

    // ---- weights ------------------------------------------------------------------------
    float4 wq[4 * kWTiles];  // tile T, k-step ks: wq[4T + ks / 4] component ks % 4
    {
        const float4* src = a.wwide + ((size_t)(w * 8 + v) * 4 * kWTiles) * 64 + l;
#pragma unroll
        for (int q = 0; q < 4 * kWTiles; ++q) wq[q] = src[(size_t)q * 64];
        const float4* hs = a.wwide_lds + (size_t)w * (WL_HH2_SZ / 4);
        float4* hd = reinterpret_cast<float4*>(lds + WL_HH2);
        for (int i = tid; i < WL_HH2_SZ / 4; i += kPT) hd[i] = hs[i];
    }
#define WR(T, ks) f4c(wq[4 * (T) + (ks) / 4], (ks) % 4)
    const float4* hh2 = reinterpret_cast<const float4*>(lds + WL_HH2);
    // ---- state and per-cell constants --------------------------------------------------
    // cell state in registers: h1, h2, x1 and gh2 = W_hh2 h2 + b_hh2 of the next GRU2 (the
    // epilogue lanes sum the gh partials themselves, in the hop D wait)
    float h1r = 0.f, h2r = 0.f, x1c = 0.f;
    float g1r = 0.f, g1z = 0.f, g1n = 0.f, g2r = 0.f, g2z = 0.f, g2n = 0.f;
    if (cell) {
        h1r = a.st_h1[(size_t)crow * kPH + cu];
        h2r = a.st_h2[(size_t)crow * kPH + cu];
        x1c = a.st_x1[(size_t)crow * kPH + cu];
        g2r = a.st_gh2[(size_t)crow * 3 * kPH + cu];
        g2z = a.st_gh2[(size_t)crow * 3 * kPH + kPH + cu];
        g2n = a.st_gh2[(size_t)crow * 3 * kPH + 2 * kPH + cu];
    }
    if (tid < R) {
        reinterpret_cast<RowInfo*>(lds + WL_RI)[tid] = a.rows[g0 + kPG * tid];
        reinterpret_cast<int2*>(lds + WL_VM)[tid] = ROT ? a.vmap[g0 + kPG * tid] : make_int2(g0 + kPG * tid, 0);
    }
    if (tid == 0) lds[WL_FAIL] = 0.f;
    // biases of the slot in LDS: read per step by the epilogues (a global load there would
    // hold up the wave's next poll behind its latency)
    if (tid < (C10 ? 128 : 112)) {
        const int k = tid < 96 ? tid % 48 : tid - 96;
        const float* src = tid < 48 ? a.b_hh1 : tid < 96 ? a.b_hh2 : a.b_fc3;
        const int cls = 16 * w + (k & 15) + (k >= 16 ? kPH : 0);  // (fc3: tile a, then tile b)
        const int idx = tid < 96 ? (k / 16) * kPH + 16 * w + (k & 15) : cls;
        lds[WL_BIAS + tid] = tid >= 96 && cls >= a.n_classes ? 0.f : src[idx];
    }
    // byte offsets in a slot: this lane's packet 0 (consumer); the packet of the unit quad
    // cul .. cul + 3 of row cn (producer: lane cul % 4 == 0 of the quad gathers and publishes;
    // slot w = wave e = w / 4, k-slot c = w % 4, packet p = cul / 4)
    const unsigned o_cons = wide::cons_off(v, l);
    const unsigned o_prod = wide::prod_off(w, cn, cul);
    // publish the cell's value of step s: slot s & 1, and the sentinel into slot (s + 1) & 1
    // every wave and lane issues the publish stores; a lane that does not publish stores to an
    // out-of-range offset (dropped by the buffer range check), so every path through a stage
    // carries the same stores and a poll issued before them need not wait for their acks
    auto pub_if = [&](bool on, int hb, float val, unsigned s) {
        const float u1 = pdpp<0x39>(val), u2 = pdpp<0x4E>(val), u3 = pdpp<0x93>(val);
        const unsigned vo = on && cell && (cul & 3) == 0 ? o_prod : wide::kNoOffset;
        __builtin_amdgcn_raw_buffer_store_b128(
            (u4v){__float_as_uint(val), __float_as_uint(u1), __float_as_uint(u2), __float_as_uint(u3)}, xr, vo,
            wide::slot_base(hb, s), 0);
        __builtin_amdgcn_raw_buffer_store_b128((u4v){kSent, kSent, kSent, kSent}, xr, vo,
                                               wide::slot_base(hb, s + 1u), 0);
    };
    auto pub = [&](int hb, float val, unsigned s) {
        // quad_perm [1,2,3,0] / [2,3,0,1] / [3,0,1,2]: quad lane 0 receives lanes 1, 2, 3
        const float u1 = pdpp<0x39>(val), u2 = pdpp<0x4E>(val), u3 = pdpp<0x93>(val);
        if (cell && (cul & 3) == 0) {
            __builtin_amdgcn_raw_buffer_store_b128(
                (u4v){__float_as_uint(val), __float_as_uint(u1), __float_as_uint(u2), __float_as_uint(u3)}, xr, o_prod,
                wide::slot_base(hb, s), 0);
            __builtin_amdgcn_raw_buffer_store_b128((u4v){kSent, kSent, kSent, kSent}, xr, o_prod,
                                                   wide::slot_base(hb, s + 1u), 0);
        }
    };
    // a cell's sums of the 8 waves' partials of tiles 0 .. K - 1 of the NT-tile buffer at P
    // (fixed order v = 0 .. 7), every LDS read issued before the first add: at this kernel's
    // register pressure the scheduler otherwise waits on the reads pair by pair
    auto psums = [&](auto kc, int P, int NT, float* out) {
        constexpr int K = decltype(kc)::value;
        float p[K][8];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int vv = 0; vv < 8; ++vv) p[k][vv] = lds[P + ((vv * NT + k) * 16 + cn) * 16 + wsw(cn, cul)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float s = 0.f;
#pragma unroll
            for (int vv = 0; vv < 8; ++vv) s += p[k][vv];
            out[k] = s;
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I3 = std::integral_constant<int, 3>;
    const rsrc_t fcr = mk_rsrc(a.fcond);
    constexpr int NC = C10 ? 32 : 16;  // noise classes per row and slot in the LDS ring
    // per-step operands of the cell, loaded right after the hop E poll (L2-resident per-frame
    // tables):
    //   pc[0..2] GRU2 cond (W_ih2[:, 512:] a2 + b_ih2), pc[3] fc1 cond, pc[4] fc2 cond (frame t)
    // and right after the hop C poll (live only from fc3 to GRU1: fewer registers held over the
    // step's products):
    //   pg (pg2) Gumbel noise of (row, class cu (512 + cu)) at step t (LDS ring, WL_GR)
    //   pp       P1(t + 1) of (row, unit cu), consumed by GRU1          (LDS ring, WL_P1R)
    //   pv       v = W_ih1 w0 (r, z, n) and w0 of unit cu         (constants, L1-resident)
    float pc[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, pg = 0.f, pg2 = 0.f;
    float4 pp = make_float4(0.f, 0.f, 0.f, 0.f), pv = make_float4(0.f, 0.f, 0.f, 0.f);
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
    };
    const rsrc_t vr = mk_rsrc(a.v), w0r = mk_rsrc(a.w0);
    auto prefetch_d = [&]() {
        if (!cell) return;
        int uu = cu;
        asm volatile("" : "+v"(uu));
        pg = lds[WL_GR + cn * NC + cul];
        if constexpr (C10) pg2 = lds[WL_GR + cn * NC + 16 + cul];
        pp = reinterpret_cast<const float4*>(lds + WL_P1R)[cn * 16 + cul];
        pv.x = bld(vr, (unsigned)uu * 4u, 0);
        pv.y = bld(vr, (unsigned)uu * 4u, kPH * 4);
        pv.z = bld(vr, (unsigned)uu * 4u, 2 * kPH * 4);
        pv.w = bld(w0r, (unsigned)uu * 4u, 0);
    };
    // The per-step operands of cell (row n, unit / class 16 w + j), formed by waves 4-7 (no
    // epilogue cells; idle while waves 0-3 run the fc3 epilogue, hop D and GRU1) into one-slot
    // LDS rings -- produced and consumed by the slot itself, so they never leave the CU (round 4
    // kept them in a 4-slot global ring whose L2 write-backs were 8 GB per C4 launch):
    //  * noise_make: the Gumbel noise of (tau, row, class) in k_gumbel's fixed-point form
    //    (philox.h gumbel_q_of) -- no [S][B][n] noise stream; formed for step t + 1 in step t's
    //    hop-D window (the slot's step-t values were read before that step's stage-D barrier);
    //  * p1_make: P1(tau) as k_persist's ring producers form it (kernels_persist.hip p1_loads /
    //    p1_store: k_p1_expand's fma chain without its zero tap) from the per-frame tables
    //    (a.p1q, runtime.hip pack_p1): the phase's 4 taps, 4 frame rows of Q and one of Aq -- no
    //    [S][B][4H] stream; with WRNN_P1_RING=0 (a.p1q null) copied from that stream instead;
    //    formed for step t + 2 in step t's hop-D window (GRU1 at the end of step t + 1 reads it).
    // (a time-sliced row at offset off: its own steps end at S, its noise is drawn at its
    // absolute step)
    auto noise_make = [&](int n, int j, int tau) {
        const int off = ROT ? reinterpret_cast<const int2*>(lds + WL_VM)[n].y : 0;
        int uu = 16 * w + j;
        asm volatile("" : "+v"(uu));
        const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + WL_RI)[n];
        // (a padding class beyond n_classes is drawn and never used)
        const U4 o = philox4x32_10((uint32_t)(uu >> 2), (uint32_t)(tau + off), (uint32_t)ri.fold, ri.stream,
                                   a.k0, a.k1);
        const uint32_t wd = (uu & 3) == 0 ? o.x : (uu & 3) == 1 ? o.y : (uu & 3) == 2 ? o.z : o.w;
        lds[WL_GR + n * NC + j] = __uint_as_float(gumbel_q_of(wd));
        if constexpr (C10) {  // and of class 512 + u
            __builtin_amdgcn_sched_barrier(0);
            const U4 o2 = philox4x32_10((uint32_t)((uu + kPH) >> 2), (uint32_t)(tau + off), (uint32_t)ri.fold,
                                        ri.stream, a.k0, a.k1);
            const uint32_t wd2 = (uu & 3) == 0 ? o2.x : (uu & 3) == 1 ? o2.y : (uu & 3) == 2 ? o2.z : o2.w;
            lds[WL_GR + n * NC + 16 + j] = __uint_as_float(gumbel_q_of(wd2));
        }
    };
    auto p1_make = [&](int n, int j, int tau) {
        const int off = ROT ? reinterpret_cast<const int2*>(lds + WL_VM)[n].y : 0;
        const int tc = tau < a.S - off ? tau : a.S - off - 1;
        int uu = 16 * w + j;
        asm volatile("" : "+v"(uu));
        const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + WL_RI)[n];
        float4 v;
        if (a.p1q == nullptr) {
            // (uniform base + 32-bit lane offset: a per-lane 64-bit address spilled)
            v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                               mk_rsrc(a.P1 + (size_t)tc * a.B * 4 * kPH),
                                               ((unsigned)(g0 + kPG * n) * 4u * kPH + (unsigned)uu * 4u) * 4u, 0, 0));
        } else {
            const unsigned p = (unsigned)(ri.rel0 + tc);
            const bool in = p < (unsigned)ri.L;  // else the zero tail pad: bias only (zero frame)
            const unsigned f = p / (unsigned)a.hop, sph = in ? p - f * (unsigned)a.hop : 0u;
            const unsigned s0 = in ? (unsigned)ri.fbase - 1u + f + (sph >= (unsigned)a.p1split ? 1u : 0u)
                                   : (unsigned)ri.fbase;
            constexpr unsigned kRow = 4u * kPH * 4u;  // bytes per frame slot
            const unsigned col = (unsigned)uu * 16u;
            const float4 tk = __builtin_bit_cast(
                float4, __builtin_amdgcn_raw_buffer_load_b128(mk_rsrc(a.p1taps), sph * 16u, 0, 0));
            const rsrc_t qr = mk_rsrc(a.p1q);
            float4 tq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                tq[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       qr, (in ? s0 + (unsigned)k : s0) * kRow + col, 0, 0));
            const float4 ta = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                             mk_rsrc(a.p1a), (in ? (unsigned)ri.fbase + 1u + f : s0) * kRow + col, 0, 0));
            float4 m = make_float4(0.f, 0.f, 0.f, 0.f);
            const float kk[4] = {tk.x, tk.y, tk.z, tk.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                m.x = fmaf(kk[k], tq[k].x, m.x);
                m.y = fmaf(kk[k], tq[k].y, m.y);
                m.z = fmaf(kk[k], tq[k].z, m.z);
                m.w = fmaf(kk[k], tq[k].w, m.w);
            }
            v = make_float4(p_add(m.x, ta.x), p_add(m.y, ta.y), p_add(m.z, ta.z), p_add(m.w, ta.w));
        }
        reinterpret_cast<float4*>(lds + WL_P1R)[n * 16 + j] = v;
    };
    const bool lo = v < 4;  // waves 0-3 hold the epilogue cells
    __syncthreads();  // RowInfo in LDS
    // ring prologue: the noise of step t0 and P1(t0 + 1) (the loop forms the noise of t + 1 and
    // P1(t + 2) at step t); the first reads come after the barrier
    if (!lo && tid - 256 < 16 * R) {
        const int i = tid - 256;
        noise_make(i >> 4, i & 15, a.t0);
        p1_make(i >> 4, i & 15, a.t0 + 1);
    }
    __syncthreads();
    // initial hop E: x1, h1 of step t0 (k_persist_init) as step t0 + 1 (canonicalised: a
    // signalling NaN in a carried state must not read as the sentinel)
    pub(WB_X1, __builtin_canonicalizef(x1c), (unsigned)a.t0 + 1u);
    pub(WB_H1, __builtin_canonicalizef(h1r), (unsigned)a.t0 + 1u);
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[0] = p_now();
    for (int t = a.t0; t < a.t1; ++t) {
        const unsigned seq = (unsigned)t + 1u;
        const unsigned so_x1 = wide::slot_base(WB_X1, seq), so_h1 = wide::slot_base(WB_H1, seq);
        const unsigned so_x2 = wide::slot_base(WB_X2, seq), so_h2 = wide::slot_base(WB_H2, seq);
        const unsigned so_y1 = wide::slot_base(WB_Y1, seq), so_y2 = wide::slot_base(WB_Y2, seq);
        u4v cc[4];
        bool fail = false;
        float x2s = 0.f;  // the value a lo wave publishes (x2, then y1)
        WSTAMP(0);
        // ================= hop E -> stage A: W_ih2[:, :512] x1 (critical) ==================
        fail |= !w_poll(xr, o_cons, so_x1, bvalid, cc, a.ctl, wh(1), (unsigned)t);
        prefetch(t);
        WSTAMP(1);
        {
            v4f acc[3] = {(v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                const float b = bop(cc, ks);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[j] = mfma4(WR(j, ks), b, acc[j]);
            }
            // PA still holds the W_hh2 h2 partials of step t - 1, which waves 0-3 read in their
            // hop D (gh2, after the candidate store). Waves 4-7 poll x1 of OTHER slots only
            // (wave v: slots 4v .. 4v + 3), so nothing orders those reads before this store but
            // a barrier: every wave reaches it after its hop-E poll anyway.
            wbar();
#pragma unroll
            for (int j = 0; j < 3; ++j)
                *reinterpret_cast<v4f*>(lds + WL_PA + ((v * 3 + j) * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc[j];
        }
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(2);
        // The step's one failure check: a wave whose poll gave up (timeout, or PC_ERR raised by
        // another slot) finishes the step on whatever its registers hold; every other poll of
        // the step ends within 64 spins of PC_ERR, so all waves come back here. (A check after
        // every stage barrier cost an LDS round trip each in front of the epilogue's reads.)
        if (lds[WL_FAIL] != 0.f) return;
        // h1 (published with x1, read above) loads now: in flight over the GRU2 epilogue, so the
        // off-path W_hh1 h1 starts without an L2 round trip
        w_issue(xr, o_cons, so_h1, bvalid, cc);
        // ================= GRU2 epilogue (waves 0-3) -> publish x2, h2 =====================
        if (lo) {
            float x2 = 0.f;
            if (cell) {
                float gi[3];
                psums(I3(), WL_PA, 3, gi);
#pragma unroll
                for (int j = 0; j < 3; ++j) gi[j] = p_add(gi[j], pc[j]);
                h2r = p_gru(gi[0], gi[1], gi[2], g2r, g2z, g2n, h2r);
                x2 = p_add(x1c, h2r);
            }
            x2s = x2;
        }
        pub_if(lo, WB_X2, x2s, seq);
        pub_if(lo, WB_H2, h2r, seq);
        WSTAMP(3);
        // ================= W_hh1 h1 -> gh1 partials (off-path, hop A wait) ==================
        {
            fail |= !w_poll(xr, o_cons, so_h1, bvalid, cc, a.ctl, wh(2), (unsigned)t, true);
            WXSTAMP(26);
            v4f acc[3] = {(v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                const float b = bop(cc, ks);
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[j] = mfma4(WR(3 + j, ks), b, acc[j]);
                // x2's first poll round, packet by packet as the h1 packets are consumed (the
                // same for y1 over W_hh2 h2 measured no gain: 125.2 against 125.5 ms per launch)
                if ((ks & 3) == 3) w_issue1(xr, o_cons, so_x2, bvalid, cc[ks >> 2], ks >> 2);
            }
#pragma unroll
            for (int j = 0; j < 3; ++j)
                *reinterpret_cast<v4f*>(lds + WL_PH + ((v * 3 + j) * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc[j];
        }
        WXSTAMP(27);
        // ================= hop A -> stage B: fc1 x2 (critical) =============================
        fail |= !w_poll(xr, o_cons, so_x2, bvalid, cc, a.ctl, wh(3), (unsigned)t, true);
        // h2 (published with x2, just read) loads now: in flight over fc1 and its epilogue
        u4v ch[4];
        w_issue(xr, o_cons, so_h2, bvalid, ch);
        WSTAMP(4);
        {
            v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 16; ks += 2) {
                acc0 = mfma4(WR(6, ks), bop(cc, ks), acc0);
                acc1 = mfma4(WR(6, ks + 1), bop(cc, ks + 1), acc1);
            }
            *reinterpret_cast<v4f*>(lds + WL_PS + (v * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc0 + acc1;
        }
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(5);
        // fc1 epilogue (waves 0-3): y1 = relu(fc1 x2 + fc1[:, 512:] a3 + b) -> publish
        if (lo) {
            float y = 0.f;
            if (cell) {
                float s;
                psums(I1(), WL_PS, 1, &s);
                y = p_add(s, pc[3]);
                y = y > 0.f ? y : 0.f;
            }
            x2s = y;
        }
        pub_if(lo, WB_Y1, x2s, seq);
        // ================= W_hh2 h2 -> gh2 partials (off-path, hop B wait) ==================
        {
            WXSTAMP(28);
            fail |= !w_poll(xr, o_cons, so_h2, bvalid, ch, a.ctl, wh(5), (unsigned)t, true);
#pragma unroll
            for (int i = 0; i < 4; ++i) cc[i] = ch[i];
            WXSTAMP(29);
            v4f acc[3] = {(v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}, (v4f){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __builtin_amdgcn_sched_barrier(0);  // one k-quad of LDS weights live at a time
                float4 aw[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) aw[j] = hh2[((j * 8 + v) * 4 + q) * 64 + l];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float b = bop(cc, 4 * q + k);
#pragma unroll
                    for (int j = 0; j < 3; ++j) acc[j] = mfma4(f4c(aw[j], k), b, acc[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < 3; ++j)
                *reinterpret_cast<v4f*>(lds + WL_PA + ((v * 3 + j) * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc[j];
        }
        WXSTAMP(30);
        // ================= hop B -> stage C: fc2 y1 (critical) =============================
        fail |= !w_poll(xr, o_cons, so_y1, bvalid, cc, a.ctl, wh(6), (unsigned)t);
        WSTAMP(6);
        {
            v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 16; ks += 2) {
                acc0 = mfma4(WR(7, ks), bop(cc, ks), acc0);
                acc1 = mfma4(WR(7, ks + 1), bop(cc, ks + 1), acc1);
            }
            *reinterpret_cast<v4f*>(lds + WL_PS + (v * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc0 + acc1;
        }
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(7);
        if (lo) {  // fc2 epilogue: y2 = relu(fc2 y1 + fc2[:, 512:] a4 + b) -> publish
            float y = 0.f;
            if (cell) {
                float s;
                psums(I1(), WL_PS, 1, &s);
                y = p_add(s, pc[4]);
                y = y > 0.f ? y : 0.f;
            }
            pub(WB_Y2, y, seq);
        }
        if constexpr (C10) {
            // gh1 = W_hh1 h1 + b_hh1 and gh2 = W_hh2 h2 + b_hh2 now (hop D without C10): PH then
            // takes the second tile's partials (written after the stage-D barrier, which every
            // wave reaches after these reads)
            if (lo && cell) {
                float gs[6];
                psums(I3(), WL_PH, 3, gs);
                psums(I3(), WL_PA, 3, gs + 3);
#pragma unroll
                for (int j = 0; j < 6; ++j) gs[j] = p_add(gs[j], lds[WL_BIAS + 16 * j + cul]);
                g1r = gs[0];
                g1z = gs[1];
                g1n = gs[2];
                g2r = gs[3];
                g2z = gs[4];
                g2n = gs[5];
            }
        }
        // ================= hop C -> stage D: fc3 y2 (critical) =============================
        fail |= !w_poll(xr, o_cons, so_y2, bvalid, cc, a.ctl, wh(8), (unsigned)t);
        // C10: the second fc3 tile's A operands of this wave (k-step ks: fb[ks / 4] component
        // ks % 4, the register tiles' order), L2-resident, in flight over the first tile
        float4 fb[4];
        if constexpr (C10) {
            const rsrc_t fr = mk_rsrc(a.wfc3b + (size_t)(w * 8 + v) * 4 * 64);
            int ll = l;
            asm volatile("" : "+v"(ll));
#pragma unroll
            for (int q = 0; q < 4; ++q)
                fb[q] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(fr, (unsigned)ll * 16u,
                                                                                         (unsigned)q * 1024u, 0));
        }
        if constexpr (!C10) prefetch_d();
        WSTAMP(8);
        {
            v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 16; ks += 2) {
                acc0 = mfma4(WR(8, ks), bop(cc, ks), acc0);
                acc1 = mfma4(WR(8, ks + 1), bop(cc, ks + 1), acc1);
            }
            *reinterpret_cast<v4f*>(lds + WL_PS + (v * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc0 + acc1;
        }
        if constexpr (C10) {
            v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 16; ks += 2) {
                acc0 = mfma4(f4c(fb[ks >> 2], ks & 3), bop(cc, ks), acc0);
                acc1 = mfma4(f4c(fb[ks >> 2], (ks + 1) & 3), bop(cc, ks + 1), acc1);
            }
            wbar();  // (every wave's gh1 / gh2 reads of PH are done)
            *reinterpret_cast<v4f*>(lds + WL_PH + (v * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc0 + acc1;
            prefetch_d();  // (after the products: fewer registers live over them)
        }
        if (fail) lds[WL_FAIL] = 1.f;
        wbar();
        WSTAMP(9);
        if (lo) {
            // fc3 epilogue: the candidate key (cand_key.h: l_k + G_k formed exactly as an fp32 pair)
            // of the slot's 16 classes per row, max over the row's DPP row of 16 lanes,
            // published with the step tag by lane cul == 0
            {
                uint32_t kh = 0, kl = 0;
                if (cell && cu < a.n_classes) {
                    float s;
                    psums(I1(), WL_PS, 1, &s);
                    const float lg = p_add(s, lds[WL_BIAS + 96 + cul]);
                    p_dbg_logit<DBG>(a.dbg, t + (ROT ? reinterpret_cast<const int2*>(lds + WL_VM)[cn].y : 0), crow, cu,
                                     a.B, a.n_classes, lg);
                    const CandKey k = cand_key(lg, __float_as_uint(pg), cu);
                    kh = k.hi;
                    kl = k.lo;
                    if constexpr (C10) {  // class 512 + cu (tile b, partials in PH)
                        if (kPH + cu < a.n_classes) {
                            float s2;
                            psums(I1(), WL_PH, 1, &s2);
                            const float lg2 = p_add(s2, lds[WL_BIAS + 112 + cul]);
                            p_dbg_logit<DBG>(a.dbg, t + (ROT ? reinterpret_cast<const int2*>(lds + WL_VM)[cn].y : 0),
                                             crow, kPH + cu, a.B, a.n_classes, lg2);
                            int c2 = kPH + cu;
                            asm volatile("" : "+v"(c2));  // (a hoisted class constant spilled)
                            const CandKey k2 = cand_key(lg2, __float_as_uint(pg2), c2);
                            kmax_take(kh, kl, k2.hi, k2.lo);
                        }
                    }
                }
                row16_kmax(kh, kl);
                if (cell && cul == 0)
                    __builtin_amdgcn_raw_buffer_store_b64((u2v){kh, kl | key_tag(seq)}, xr, wide::cand_off(cn, w),
                                                          WX_D * 4, 0);
            }
            // gh1 = W_hh1 h1 + b_hh1 (for GRU1 below) and gh2 = W_hh2 h2 + b_hh2 (the next GRU2)
            // from the off-path partials, while the candidates travel: every wave wrote them
            // before the stage C barrier. PH is rewritten in the next hop-A wait, after the next
            // stage-A barrier; PA in the next stage A behind a barrier of its own (see there):
            // this wave reaches both only after these reads have completed. (C10: read in the
            // hop-C wait, see there)
            if (!C10 && cell) {
                float gs[6];
                psums(I3(), WL_PH, 3, gs);
                psums(I3(), WL_PA, 3, gs + 3);
#pragma unroll
                for (int j = 0; j < 6; ++j) gs[j] = p_add(gs[j], lds[WL_BIAS + 16 * j + cul]);
                g1r = gs[0];
                g1z = gs[1];
                g1n = gs[2];
                g2r = gs[3];
                g2z = gs[4];
                g2n = gs[5];
            }
            // ============= hop D: sample of step t, per cell wave for its own 4 rows ========
            // lane (row cn, cul) reads the candidates of slots 2 cul, 2 cul + 1 of its row; the
            // row's 16 lanes reduce them (DPP), so every cell of the row holds the sample
            float x;
            {
                const unsigned want = key_tag(seq);
                u4v q = {0u, want, 0u, want};
                const unsigned t0s = p_now();
                unsigned nsp = 0;
                while (true) {
                    if (cell) {
                        unsigned vo = wide::cand_off(cn, 2 * cul);
                        asm volatile("" : "+v"(vo));
                        q = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, WX_D * 4, kCpNT);
                    }
                    if (__all((q.y & kKeyTagMask) == want && (q.w & kKeyTagMask) == want)) break;
                    if ((++nsp & 63) == 0 && (ld_sc1_u(a.ctl + PC_ERR) || p_now() - t0s > kSpinTicks)) {
                        if (l == 0 && !ld_sc1_u(a.ctl + PC_ERR) &&
                            atomicCAS(a.ctl + PC_WHERE, 0u, wh(9) | ((unsigned)v << 19)) == 0u)
                            a.ctl[PC_WHERE + 2] = (unsigned)t;
                        if (l == 0) atomicMax(a.ctl + PC_ERR, 2u);
                        fail = true;
                        break;
                    }
                }
                uint32_t bh = q.x, bl = q.y;
                kmax_take(bh, bl, q.z, q.w);
                row16_kmax(bh, bl);
                const int bi = key_cls(bl);
                {
#pragma clang fp contract(off)
                    x = (2.0f * (float)bi) / (float)(a.n_classes - 1) - 1.0f;
                }
                if (w == 0 && cell && cul == 0) {
                    int nn = cn;
                    asm volatile("" : "+v"(nn));
                    const int2 vm = reinterpret_cast<const int2*>(lds + WL_VM)[nn];
                    const unsigned ro = (unsigned)(vm.x * a.ld + vm.y);
                    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bi, mk_rsrc(a.labels), ro * 2u,
                                                          (unsigned)t * 2u, 0);
                    bst(x, mk_rsrc(a.samples), ro * 4u, (unsigned)t * 4u);
                }
            }
            if (fail) lds[WL_FAIL] = 1.f;  // seen by every wave at the next stage-A check
            WSTAMP(10);
            // ============= GRU1 of step t + 1 for the slot's units -> publish x1, h1 ========
            //   gi = W_ih1 (cI + w0 x) + b_ih1 = P1 + v x ; x1 = (cI + w0 x) + h1
            // (at the last step it runs on clamped inputs and nobody reads the result)
            float x1 = 0.f;
            if (cell) {
                h1r = p_gru(fmaf(pv.x, x, pp.x), fmaf(pv.y, x, pp.y), fmaf(pv.z, x, pp.z), g1r, g1z, g1n, h1r);
                x1 = p_add(fmaf(pv.w, x, pp.w), h1r);
                x1c = x1;
            }
            pub(WB_X1, x1, seq + 1u);
            pub(WB_H1, h1r, seq + 1u);
        } else {
            // waves 4-7: the noise of step t + 1 and P1(t + 2) for cell i = tid - 256 into the
            // one-slot LDS rings (waves 0-3 read the slots' step-t / P1(t + 1) values in
            // prefetch_d, before this step's stage-D barrier, and the new ones after the next
            // step's stage-A barrier)
            const int i = tid - 256;
            if (i < 16 * R) {
                noise_make(i >> 4, i & 15, t + 1);
                p1_make(i >> 4, i & 15, t + 2);
            }
        }
        if (w == 0 && tid == 0) {
            if (g == 0) p_progress(a.progress, a.prog_base, t);
            if (p_abort(a.ctl, a.progress, t)) lds[WL_FAIL] = 1.f;  // seen at the next stage-A check
        }
        WSTAMP(11);
    }
#undef WSTAMP
#undef WXSTAMP
#undef WR
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[1] = p_now();
    // ---- the rows' state for a later launch (time-sliced or chunked calls): x1, h1 of step t1
    // (GRU1 of the last step), h2 of step t1 - 1, gh2 = W_hh2 h2 + b_hh2 of the next GRU2 --
    // k_persist's chunk-state layout
    // (the row re-read from LDS: keeping crow live across the step loop cost a spilled register)
    if ((ROT || a.t1 < a.S) && cell && lds[WL_FAIL] == 0.f) {
        int nn = cn;
        asm volatile("" : "+v"(nn));
        const int row = reinterpret_cast<const int2*>(lds + WL_VM)[nn].x;
        a.st_x1[(size_t)row * kPH + cu] = x1c;
        a.st_h1[(size_t)row * kPH + cu] = h1r;
        a.st_h2[(size_t)row * kPH + cu] = h2r;
        a.st_gh2[(size_t)row * 3 * kPH + cu] = g2r;
        a.st_gh2[(size_t)row * 3 * kPH + kPH + cu] = g2z;
        a.st_gh2[(size_t)row * 3 * kPH + 2 * kPH + cu] = g2n;
    }
}

size_t persist_wide_lds_bytes() { return (size_t)WL_TOTAL * sizeof(float); }
size_t persist_wide_xbuf_floats() { return (size_t)kPG * WX_GROUP; }
// before every wide launch: the vector slots to the sentinel, the candidate area (step tags) to 0
__global__ __launch_bounds__(256) void k_wide_xbuf_reset(uint4* x) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)kPG * WX_GROUP / 4) return;
    const unsigned f = (unsigned)((i * 4) % WX_GROUP);
    x[i] = f >= (unsigned)WX_D ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(kSent, kSent, kSent, kSent);
}
hipError_t persist_wide_reset_xbuf(float* xbuf, hipStream_t s) {
    const unsigned n = (unsigned)((size_t)kPG * WX_GROUP / 4);
    k_wide_xbuf_reset<<<(n + 255) / 256, 256, 0, s>>>(reinterpret_cast<uint4*>(xbuf));
    return hipGetLastError();
}
size_t persist_wide_ring_floats() { return 64; }  // (no global ring since round 5: LDS rings)

// Exhaustive host-side check of the exchange layout for a group of R rows (wide_layout.h): the
// producer packets of one hop slot (32 slots x R rows x 4 unit quads) and the consumer packets
// (8 waves x 64 lanes x 4 packets, lanes of rows >= R off) are the same set, each once, every
// matched pair carries the same (row, unit quad), all 16-byte aligned inside the slot's main
// region; slots of different buffers / parities never overlap; the candidates fit their area;
// the no-packet offset fails the range check for every slot base. Returns the violations.
int wide_layout_check(int R) {
    using namespace wide;
    if (R < 1 || R > kRows) return -1;
    int bad = 0;
    std::vector<int> owner(WS_MAIN / 4, -1);  // packet index -> producer id
    for (int w = 0; w < kSlots; ++w)
        for (int cn = 0; cn < R; ++cn)
            for (int cul = 0; cul < 16; cul += 4) {
                const unsigned o = prod_off(w, cn, cul);
                if (o % 16 || o + 16 > (unsigned)WS_MAIN * 4u) { ++bad; continue; }
                int& ow = owner[o / 16];
                if (ow >= 0) ++bad;  // two producers on one packet
                ow = (w * kRows + cn) * 16 + cul;
            }
    int matched = 0;
    for (int v = 0; v < kWaves; ++v)
        for (int l = 0; l < 64; ++l) {
            if (cons_row(l) >= R) continue;  // polls kNoOffset (w_issue)
            for (int i = 0; i < kPackets; ++i) {
                const unsigned o = cons_off(v, l) + 1024u * (unsigned)i;
                if (o % 16 || o + 16 > (unsigned)WS_MAIN * 4u) { ++bad; continue; }
                const int ow = owner[o / 16];
                if (ow < 0) { ++bad; continue; }  // nobody publishes what this lane waits for
                const int w = ow / (kRows * 16), cn = (ow / 16) % kRows, cul = ow % 16;
                if (cn != cons_row(l) || 16 * w + cul != cons_unit0(v, l, i)) ++bad;
                ++matched;
            }
        }
    if (matched != kSlots * R * 4) ++bad;  // a publication nobody reads
    // buffer / parity slots: disjoint, inside [0, WX_D); the candidate area after them
    for (int hb = 0; hb < kBufs; ++hb)
        for (unsigned s = 0; s < 2; ++s) {
            const unsigned b = slot_base(hb, s);
            if (b != (unsigned)(hb * 2 + (int)s) * (unsigned)WSLOT * 4u) ++bad;
            if (b + (unsigned)WSLOT * 4u > (unsigned)WX_D * 4u) ++bad;
            if ((unsigned long long)kNoOffset + b + 1024ull * kPackets <= kRsrcRecords) ++bad;
        }
    for (int n = 0; n < R; ++n)
        for (int w = 0; w < kSlots; w += 2)
            if (cand_off(n, w) + 16 > (unsigned)WX_CAND * 4u || cand_off(n, w) % 16) ++bad;
    return bad;
}
size_t persist_wide_wreg_floats() { return (size_t)kPM * 8 * 4 * kWTiles * 64 * 4; }
size_t persist_wide_wlds_floats() { return (size_t)kPM * WL_HH2_SZ; }

int persist_wide_scratch(bool c10) {
    hipFuncAttributes fa;
    const void* f = c10 ? (const void*)k_persist_wide<false, true, false> : (const void*)k_persist_wide<false, false, false>;
    if (hipFuncGetAttributes(&fa, f) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}
int persist_wide_rot_scratch(bool c10) {
    hipFuncAttributes fa;
    const void* f = c10 ? (const void*)k_persist_wide<true, true, false> : (const void*)k_persist_wide<true, false, false>;
    if (hipFuncGetAttributes(&fa, f) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}

hipError_t launch_persist_wide(const PersistArgs& a, hipStream_t s) {
    if (a.rb < 0 || a.nr < 1 || a.nr > kPWideRows || a.rb + kPG * a.nr > a.B || a.n_classes > 2 * kPM * 16 ||
        a.mode != 0 || a.wwide == nullptr || (a.n_classes > kPM * 16 && a.wfc3b == nullptr))
        return hipErrorInvalidValue;
    const size_t lb = persist_wide_lds_bytes();
    const bool dbg = a.dbg.out != nullptr;
    if (a.vmap && a.p1q == nullptr) return hipErrorInvalidValue;  // time-sliced rows: P1 formed in-kernel
    if (a.n_classes > kPM * 16) {
        if (a.vmap) return dbg ? persist_launch<k_persist_wide<true, true, true>>(lb, a, s)
                               : persist_launch<k_persist_wide<true, true, false>>(lb, a, s);
        return dbg ? persist_launch<k_persist_wide<false, true, true>>(lb, a, s)
                   : persist_launch<k_persist_wide<false, true, false>>(lb, a, s);
    }
    if (a.vmap) return dbg ? persist_launch<k_persist_wide<true, false, true>>(lb, a, s)
                           : persist_launch<k_persist_wide<true, false, false>>(lb, a, s);
    return dbg ? persist_launch<k_persist_wide<false, false, true>>(lb, a, s)
               : persist_launch<k_persist_wide<false, false, false>>(lb, a, s);
}

}  // namespace wrnn
