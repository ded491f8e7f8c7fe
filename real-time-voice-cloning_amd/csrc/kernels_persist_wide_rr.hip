// Persistent runtimeracer recurrence for WIDE row batches (launch kind "persist-wide" of the
// runtimeracer topology): up to 16 fold rows per XCD group, 128 rows per launch, every product
// on the fp32 matrix cores (v_mfma_f32_16x16x4_f32).
//
// Reference step body: vocoder/models/runtimeracer_version.py:244-270 (rnn_dims = fc_dims = 256):
//   x1 = I(x0) + h1'          h1' = rnn1(I(x0), h1)
//   x2 = x1 + rnn2(x1, h2)    x3 = x2 + rnn3([x2, a2], h3)    x4 = x3 + rnn4(x3, h4)
//   y1 = fc1([x4, a3])        y2 = relu(fc2(y1))    y3 = fc3([y2, a4])    y4 = relu(fc4(y3))
//   logits = fc5(y4) -> categorical draw
// restructured as kernels_persist_rr.hip (conditioning per frame, P1 + v x for GRU1's input).
//
// Layout: the 32 workgroups of an XCD group form two HALVES of 16 slots; slot s of a half owns
// units [16 s, 16 s + 16) of ITS half's layers, so every MFMA tile is a full 16-row M tile
// (8 units per slot of every layer, the register-resident kernel's split, would leave tiles
// half empty):
//   half A (slots 0-15):  GRU2 (W_ih2, W_hh2), GRU4 (W_ih4, W_hh4), fc2, fc4
//   half B (slots 16-31): GRU1 (W_hh1; its input term is P1 + v x), GRU3 (W_ih3[:, :256],
//                         W_hh3), fc1[:, :256], fc3[:, :256], fc5 (n / 16 classes per slot)
// The step is a ping-pong of nine hops between the halves, each half computing while the other
// waits for its vector:
//   B: GRU1 -> x1 | A: GRU2 -> x2 | B: GRU3 -> x3 | A: GRU4 -> x4 | B: fc1 -> y1 | A: fc2 -> y2
//   B: fc3 -> y3 | A: fc4 -> y4 | B: fc5 -> per-slot candidates -> (B) sample + GRU1 ...
// and the recurrent products run in the half's waits: A's W_hh2 h2 while B runs GRU3, W_hh4 h4
// while B runs fc1; B's W_hh1 h1 while A runs GRU2, W_hh3 h3 while A runs GRU4. A forms its
// partner B slot's P1 and Gumbel noise three steps ahead (per-slot ring in L2) while B runs fc5,
// the sample and GRU1.
// K = 256 is split over the 8 waves (wave v: inputs [32 v, 32 v + 32), 8 k-steps of 4), the 8
// partial tiles summed in LDS in a fixed order by the epilogue lanes (256 cells = 16 rows x 16
// units on waves 0-3). Vectors are exchanged as 16-byte packets in MFMA B-operand order (two per
// consumer lane and hop), untagged with a sentinel-reset slot pair per vector (the protocol of
// kernels_persist_wide.hip) -- consumer and producer halves alternate, so every
// consumer has read a later publication of each producer wave before it polls the reset slot.
#include "wrnn_kernels.h"
#include "persist_common.h"
#include "philox.h"

#include <vector>

namespace wrnn {
namespace {

typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int RH = kRH;        // 256
constexpr int kHalf = 16;      // slots per half
constexpr int kRowsW = 16;     // rows per group (MFMA N)
constexpr unsigned kSentR = 0x7fbadbadu;  // a signalling NaN: no arithmetic result is ever this
constexpr unsigned kNoOff = 0x80000000u;  // lanes without a packet: outside every buffer

// ---- exchange area per group (floats) ---------------------------------------------------
// one vector per step and parity slot: [e 8][p 2][lane 64] packets of 4 floats; packet p of
// consumer lane l = 16 c + n of wave e holds row n, units 32 e + 8 c + 4 p + q (q < 4)
constexpr int QSLOT = 8 * 2 * 64 * 4;
constexpr int QV = 2 * QSLOT;
enum QBuf : int { QX1 = 0, QH1, QX2, QH2, QX3, QH3, QX4, QH4, QY1, QY2, QY3, QY4, QN };
constexpr int QX_D = QN * QV;  // candidates [row 16][B slot 16] (value, step tag << 11 | class)
constexpr int QX_GROUP = QX_D + kRowsW * kHalf * 2 + 64;
static_assert(QX_GROUP % 4 == 0 && QX_D % 4 == 0, "reset works in 16-byte units");

__host__ __device__ constexpr unsigned q_cons(int v, int l) { return (unsigned)((v * 2 * 64 + l) * 16); }
// packet of the unit quad u .. u + 3 (u = 16 s + cul, cul % 4 == 0) of row cn
__host__ __device__ constexpr unsigned q_prod(int s, int cn, int cul) {
    return (unsigned)(((((16 * s + cul) >> 5) * 2 + (((16 * s + cul) >> 2) & 1)) * 64 +
                       16 * (((16 * s + cul) >> 3) & 3) + cn) * 16);
}
__host__ __device__ constexpr unsigned q_slot(int hb, unsigned seq) {
    return (unsigned)(hb * QV) * 4u + (seq & 1u) * (unsigned)QSLOT * 4u;
}
__host__ __device__ constexpr unsigned q_cand(int n, int s) { return (unsigned)((n * kHalf + s) * 2) * 4u; }

// ---- per-slot operand ring (PersistRRArgs::wring): for B slot s, written by A slot s --------
// [4 step slots][16 rows][16 units] float4 P1 (r, z, n of W_ih1 (I c) + b_ih1, then I c + b_I),
// then [4][16 rows][64 classes] float Gumbel noise
constexpr int RG_P = 4 * kRowsW * 16 * 4;
constexpr int RG_SLOT = RG_P + 4 * kRowsW * 64;

// ---- LDS (floats) -------------------------------------------------------------------------
constexpr int QL_RI = 0;         // RowInfo of the group's rows (6 words each)
constexpr int QL_FAIL = 112;
constexpr int QL_REG = 116;      // group, slot, registration result (ints)
constexpr int QL_CB = 128;       // slot constants (biases), see the halves (<= 224 floats)
constexpr int QL_VM = 448;       // (physical row, step offset) of each row slot (int2, ROT)
constexpr int QL_P = 512;        // partial tiles [8 v][nt][16 n][16 m], one buffer per product
constexpr int T3 = 8 * 3 * 256, T1 = 8 * 256;
// half A
constexpr int PA_G2 = QL_P, PA_H2 = PA_G2 + T3, PA_G4 = PA_H2 + T3, PA_H4 = PA_G4 + T3,
              PA_F2 = PA_H4 + T3, PA_F4 = PA_F2 + T1, PA_END = PA_F4 + T1;
// half B
constexpr int PB_H1 = QL_P, PB_G3 = PB_H1 + T3, PB_H3 = PB_G3 + T3, PB_F1 = PB_H3 + T3,
              PB_F3 = PB_F1 + T1, PB_F5 = PB_F3 + T1, PB_END = PB_F5 + 4 * T1;
constexpr int QL_TOTAL = PA_END > PB_END ? PA_END : PB_END;
static_assert(QL_TOTAL * 4 <= 160 * 1024, "LDS carve exceeds the CU's 160 KiB");
static_assert(sizeof(RowInfo) == 24 && kRowsW * 6 <= QL_FAIL, "RowInfo array overflows");
static_assert(QL_CB + 224 <= QL_VM && QL_VM + 2 * kRowsW <= QL_P, "small LDS arrays overflow");

constexpr int kWq = 30;  // float4 weight registers per lane: 15 tiles x 8 k-steps

__device__ __forceinline__ v4f mfma4(float a, float b, v4f c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float f4c(const float4& q, int i) {
    return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
}
__device__ __forceinline__ float bop2(const u4v (&cc)[2], int ks) {
    const u4v& q = cc[ks >> 2];
    return __uint_as_float((ks & 3) == 0 ? q.x : (ks & 3) == 1 ? q.y : (ks & 3) == 2 ? q.z : q.w);
}
// conflict-free partial tiles: XOR swizzle of the 16-byte column slots by row (as the
// fatchord wide kernel, kernels_persist_wide.hip wsw)
__device__ __forceinline__ int wsw(int n, int o) { return ((((o >> 2) ^ (n >> 1)) & 3) << 2) | (o & 3); }
__device__ __forceinline__ bool q_ready(const u4v& q) {
    return (q.x != kSentR) & (q.y != kSentR) & (q.z != kSentR) & (q.w != kSentR);
}
__device__ __forceinline__ void qbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// One poll round of a hop: the lane's 2 B-operand packets and (cell lanes) the 4-byte value of
// its own cell (own == kNoOff: none). Lanes without a packet load from kNoOff (reads 0).
__device__ __forceinline__ void q_issue(rsrc_t xr, unsigned voff, unsigned so, bool valid, unsigned own,
                                        u4v (&cc)[2], unsigned& ov) {
    unsigned vo = valid ? voff : kNoOff;
    asm volatile("" : "+v"(vo));
    cc[0] = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, so, kCpNT);
    cc[1] = __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 1024u, so, kCpNT);
    ov = __builtin_amdgcn_raw_buffer_load_b32(xr, own, so, kCpNT);
}
// Poll until no value is the sentinel (see kernels_persist_wide.hip w_poll for the protocol);
// bounded, records the first timeout's site like the fatchord wide kernel.
__device__ __forceinline__ bool q_poll(rsrc_t xr, unsigned voff, unsigned so, bool valid, unsigned own,
                                       u4v (&cc)[2], unsigned& ov, unsigned* ctl, unsigned where,
                                       unsigned step) {
    const unsigned t0 = p_now();
    unsigned nsp = 0;
    while (true) {
        q_issue(xr, voff, so, valid, own, cc, ov);
        if (__all((int)q_ready(cc[0]) & (int)q_ready(cc[1]) & (int)(ov != kSentR))) return true;
        if ((++nsp & 63) == 0 && (ld_sc1_u(ctl + PC_ERR) || p_now() - t0 > kSpinTicks)) {
            if ((threadIdx.x & 63) == 0 && !ld_sc1_u(ctl + PC_ERR) &&
                atomicCAS(ctl + PC_WHERE, 0u, where | ((threadIdx.x >> 6) << 19)) == 0u) {
                ctl[PC_WHERE + 1] = 1u;
                ctl[PC_WHERE + 2] = step;
            }
            if ((threadIdx.x & 63) == 0) atomicMax(ctl + PC_ERR, 2u);
            return false;
        }
    }
}

}  // namespace

// DBG: the instance that records logits for the teacher-forced gate (wrnn_set_debug_steps)
// ROT: a time-sliced launch (PersistRRArgs::vmap): row slot r of group g is the
//      virtual row g + 8 r -> (physical row, step offset); the launch runs steps [0, t1) of its
//      rows (their steps off .. off + t1 - 1) from the chunk state and saves it at the end
template <bool ROT, bool DBG>
__global__ __launch_bounds__(kPT, 1) void k_persist_wide_rr(PersistRRArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    int* sreg = reinterpret_cast<int*>(lds + QL_REG);
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
    const int v = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave: inputs [32 v, 32 v + 32)
    const int l = tid & 63;
    const int half = w >> 4, s = w & 15;
    const int R = a.nr;
    const int g0 = a.rb + g;
    const int bn = l & 15;
    const bool bvalid = bn < R;
    const int cn = tid >> 4, cul = tid & 15;  // epilogue cell (row cn, unit 16 s + cul), waves 0-3
    const bool cell = tid < 16 * R;
    const int cu = 16 * s + cul;
    const int crow = ROT ? a.vmap[g0 + kPG * (cell ? cn : 0)].x : g0 + kPG * (cell ? cn : 0);
    // a row slot's step offset (time-sliced launches; 0 otherwise)
    auto roff = [&](int n) { return ROT ? reinterpret_cast<const int2*>(lds + QL_VM)[n].y : 0; };
    const rsrc_t xr = mk_rsrc(a.xbuf + (size_t)g * QX_GROUP);
    const rsrc_t rgr = mk_rsrc(a.wring + ((size_t)g * kHalf + s) * RG_SLOT);  // slot s's ring
    const unsigned o_cons = q_cons(v, l);
    const unsigned o_prod = q_prod(s, cell ? cn : 0, cul & ~3);
    // own cell value of a vector published by the same-numbered slot of the other half
    const unsigned o_own = cell ? o_prod + 4u * (unsigned)(cul & 3) : kNoOff;
    auto wh = [&](unsigned site) { return site << 28 | (unsigned)w << 22; };
    const int ntc = a.cpw / 16;  // fc5 tiles of a B slot (cpw = n / 16 classes: 2 or 4)
    // phase stamps of the traced step (WRNN_PHASE_STEP), wave 0 of slots 0 (A) and 16 (B)
    uint32_t* ph = a.phases != nullptr && (w == 0 || w == 16) ? a.phases + (size_t)(g * kPM + w) * kPPhases : nullptr;
#define RS(i) \
    if (ph != nullptr && t == a.phase_t && tid == 0) ph[(i)] = p_now();

    // ---- weights: tile T, k-step ks at wq[2 T + ks / 4] component ks % 4 --------------------
    float4 wq[kWq];
    {
        const float4* src = a.wwide + ((size_t)(w * 8 + v) * kWq) * 64 + l;
#pragma unroll
        for (int q = 0; q < kWq; ++q) wq[q] = src[(size_t)q * 64];
    }
#define QW(T, ks) f4c(wq[2 * (T) + (ks) / 4], (ks) % 4)
    if (tid < R) {
        reinterpret_cast<RowInfo*>(lds + QL_RI)[tid] = a.rows[g0 + kPG * tid];
        if (ROT) reinterpret_cast<int2*>(lds + QL_VM)[tid] = a.vmap[g0 + kPG * tid];
    }
    if (tid == 0) lds[QL_FAIL] = 0.f;

    // publish the cell's value of step seq: slot seq & 1, the sentinel into slot (seq + 1) & 1
    // Every lane of the wave issues both stores (a lane that does not publish uses kNoOff, which
    // the buffer range check drops): no branch around them, so the compiler's waits after them
    // stay counted (the fatchord wide kernel's round-3 lesson)
    auto pub = [&](int hb, float val, unsigned seq) {
        const float u1 = pdpp<0x39>(val), u2 = pdpp<0x4E>(val), u3 = pdpp<0x93>(val);
        unsigned vo = cell && (cul & 3) == 0 ? o_prod : kNoOff;
        asm volatile("" : "+v"(vo));
        __builtin_amdgcn_raw_buffer_store_b128(
            (u4v){__float_as_uint(val), __float_as_uint(u1), __float_as_uint(u2), __float_as_uint(u3)}, xr, vo,
            q_slot(hb, seq), 0);
        __builtin_amdgcn_raw_buffer_store_b128((u4v){kSentR, kSentR, kSentR, kSentR}, xr, vo,
                                               q_slot(hb, seq + 1u), 0);
    };
    // NT-tile product over a hop's packets into the partial tiles at P (tiles T0 ..)
    auto prod = [&](auto ntc_, int T0, const u4v (&cc)[2], int P) {
        constexpr int NT = decltype(ntc_)::value;
        v4f acc[NT];
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const float b = bop2(cc, ks);
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[j] = mfma4(QW(T0 + j, ks), b, acc[j]);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j)
            *reinterpret_cast<v4f*>(lds + P + ((v * NT + j) * 16 + bn) * 16 + wsw(bn, 4 * (l >> 4))) = acc[j];
    };
    // a cell's sums of the 8 waves' partials of tiles j0 .. j0 + K - 1 (fixed order v = 0 .. 7),
    // every LDS read issued before the first add: at this kernel's register pressure the
    // scheduler otherwise waits on each read in turn (one LDS latency per partial)
    auto psums = [&](auto kc, int P, int NT, int j0, float* out) {
        constexpr int K = decltype(kc)::value;
        float p[K][8];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int vv = 0; vv < 8; ++vv) p[k][vv] = lds[P + ((vv * NT + j0 + k) * 16 + cn) * 16 + wsw(cn, cul)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float acc = 0.f;
#pragma unroll
            for (int vv = 0; vv < 8; ++vv) acc += p[k][vv];
            out[k] = acc;
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    bool fail = false;
    u4v cc[2];
    unsigned ov = 0;
    const unsigned o_own_none = kNoOff;

    if (half == 0) {
        // =============================== half A ===================================
        // slot constants: b_ih2, b_hh2, b_ih4, b_hh4 [3][16] each, b_f2, b_f4 [16]
        if (tid < 224) {
            const int k = tid % 48, gt = k / 16, ul = k & 15;
            const float* src = tid < 48 ? a.b_ih2 : tid < 96 ? a.b_hh2 : tid < 144 ? a.b_ih4
                               : tid < 192 ? a.b_hh4 : (tid < 208 ? a.b_f2 : a.b_f4);
            lds[QL_CB + tid] = tid < 192 ? src[gt * RH + 16 * s + ul] : src[16 * s + (tid & 15)];
        }
        float h2r = 0.f, h4r = 0.f;
        float g2r = 0.f, g2z = 0.f, g2n = 0.f, g4r = 0.f, g4z = 0.f, g4n = 0.f;
        const float* cb = lds + QL_CB;
        __syncthreads();
        if (cell && !ROT) {  // h2 = h4 = 0 at step 0: gh = W_hh 0 + b_hh
            g2r = cb[48 + cul];
            g2z = cb[64 + cul];
            g2n = cb[80 + cul];
            g4r = cb[144 + cul];
            g4z = cb[160 + cul];
            g4n = cb[176 + cul];
        }
        if (cell && ROT) {  // the row's chunk state (k_persist_rr_init or an earlier slice)
            const float* st = a.st + (size_t)crow * kRRState * RH;
            h2r = st[2 * RH + cu];
            h4r = st[4 * RH + cu];
            g2r = st[5 * RH + cu];
            g2z = st[6 * RH + cu];
            g2n = st[7 * RH + cu];
            g4r = st[11 * RH + cu];
            g4z = st[12 * RH + cu];
            g4n = st[13 * RH + cu];
        }
        // the partner B slot's ring entry of step tau: thread tid < 256 forms P1 of cell
        // (row tid / 16, unit 16 s + tid % 16); thread 256 + i the Gumbel noise of classes
        // cpw s + 4 (i % 16) .. + 3 of row i / 16 (one Philox call, four words)
        auto ring_make = [&](int tau) {
            int tx = tid;
            asm volatile("" : "+v"(tx));
            if (tx < 256) {
                const int n = tx >> 4, uu = 16 * s + (tx & 15);
                if (n >= R) return;
                // (a time-sliced row: its own steps end at S)
                const int tc = tau < a.S - roff(n) ? tau : a.S - roff(n) - 1;
                const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + QL_RI)[n];
                float4 vv;
                if (a.p1q == nullptr) {
                    vv = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                        mk_rsrc(a.P1 + ((size_t)tc * a.B + g0 + kPG * n) * 4 * RH),
                                                        (unsigned)uu * 16u, 0, 0));
                } else {
                    const unsigned p = (unsigned)(ri.rel0 + tc);
                    const bool in = p < (unsigned)ri.L;  // else the zero tail pad: bias only
                    const unsigned f = p / (unsigned)a.hop, sph = in ? p - f * (unsigned)a.hop : 0u;
                    const unsigned s0 = in ? (unsigned)ri.fbase - 1u + f + (sph >= (unsigned)a.p1split ? 1u : 0u)
                                           : (unsigned)ri.fbase;
                    constexpr unsigned kRow = 4u * RH * 4u;  // bytes per frame slot
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
                    vv = make_float4(p_add(m.x, ta.x), p_add(m.y, ta.y), p_add(m.z, ta.z), p_add(m.w, ta.w));
                }
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(u4v, vv), rgr, (unsigned)(((tau & 3) * kRowsW + n) * 16 + (tx & 15)) * 16u, 0, 0);
            } else {
                const int i = tx - 256, n = i >> 4, jq = i & 15;
                if (n >= R || 4 * jq >= a.cpw) return;
                const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + QL_RI)[n];
                const int c0 = a.cpw * s + 4 * jq;  // classes c0 .. c0 + 3 (cpw % 4 == 0)
                // (drawn at the row's absolute step)
                const U4 o = philox4x32_10((uint32_t)(c0 >> 2), (uint32_t)(tau + roff(n)), (uint32_t)ri.fold,
                                           ri.stream, a.k0, a.k1);
                const u4v gv = {gumbel_q_of(o.x), gumbel_q_of(o.y), gumbel_q_of(o.z), gumbel_q_of(o.w)};
                __builtin_amdgcn_raw_buffer_store_b128(
                    gv, rgr, (unsigned)(RG_P + ((tau & 3) * kRowsW + n) * 64 + 4 * jq) * 4u, 0, 0);
            }
        };
        // ring prologue: steps t0 .. t0 + 2 (the loop forms t + 3 at step t); B reads them only
        // after polling this slot's later publications, which follow these drained stores
        for (int k = 0; k < 3; ++k) ring_make(a.t0 + k);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[0] = p_now();
        for (int t = a.t0; t < a.t1; ++t) {
            const unsigned seq = (unsigned)t + 1u;
            RS(0);
            // ---- A1: x1 -> W_ih2 x1 -> GRU2 -> x2, h2 -------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QX1, seq), bvalid, o_own, cc, ov, a.ctl, wh(1), (unsigned)t);
            RS(1);
            const float x1v = __uint_as_float(ov);
            prod(I3(), 0, cc, PA_G2);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            RS(2);
            if (lds[QL_FAIL] != 0.f) return;
            {
                float x2 = 0.f;
                if (cell) {
                    float ps[3];
                    psums(I3(), PA_G2, 3, 0, ps);
                    const float gi0 = p_add(ps[0], cb[cul]);
                    const float gi1 = p_add(ps[1], cb[16 + cul]);
                    const float gi2 = p_add(ps[2], cb[32 + cul]);
                    h2r = p_gru(gi0, gi1, gi2, g2r, g2z, g2n, h2r);
                    x2 = p_add(x1v, h2r);
                }
                if (v < 4) {
                    pub(QX2, x2, seq);
                    pub(QH2, h2r, seq);
                }
            }
            RS(3);
            // ---- A2: h2 of every A slot -> W_hh2 h2 (next step's gh2; B runs GRU3) ----------
            fail |= !q_poll(xr, o_cons, q_slot(QH2, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(2), (unsigned)t);
            RS(4);
            prod(I3(), 3, cc, PA_H2);
            RS(5);
            // ---- A3: x3 -> W_ih4 x3 -> GRU4 -> x4, h4 --------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QX3, seq), bvalid, o_own, cc, ov, a.ctl, wh(3), (unsigned)t);
            RS(6);
            const float x3v = __uint_as_float(ov);
            prod(I3(), 6, cc, PA_G4);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            {
                float x4 = 0.f;
                if (cell) {
                    float ps[3];
                    psums(I3(), PA_G4, 3, 0, ps);
                    const float gi0 = p_add(ps[0], cb[96 + cul]);
                    const float gi1 = p_add(ps[1], cb[112 + cul]);
                    const float gi2 = p_add(ps[2], cb[128 + cul]);
                    h4r = p_gru(gi0, gi1, gi2, g4r, g4z, g4n, h4r);
                    x4 = p_add(x3v, h4r);
                }
                if (v < 4) {
                    pub(QX4, x4, seq);
                    pub(QH4, h4r, seq);
                }
                if (cell) {
                    float ps[3];
                    psums(I3(), PA_H2, 3, 0, ps);
                    g2r = p_add(ps[0], cb[48 + cul]);
                    g2z = p_add(ps[1], cb[64 + cul]);
                    g2n = p_add(ps[2], cb[80 + cul]);
                }
            }
            RS(7);
            // ---- A4: h4 of every A slot -> W_hh4 h4 (next step's gh4; B runs fc1) -----------
            fail |= !q_poll(xr, o_cons, q_slot(QH4, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(4), (unsigned)t);
            prod(I3(), 9, cc, PA_H4);
            RS(8);
            // ---- A5: y1 -> fc2 -> y2 --------------------------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QY1, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(5), (unsigned)t);
            RS(9);
            prod(I1(), 12, cc, PA_F2);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            {
                float y = 0.f;
                if (cell) {
                    float ps[3];
                    psums(I1(), PA_F2, 1, 0, ps);
                    y = p_add(ps[0], cb[192 + cul]);
                    y = y > 0.f ? y : 0.f;
                }
                if (v < 4) pub(QY2, y, seq);
                if (cell) {
                    float ps[3];
                    psums(I3(), PA_H4, 3, 0, ps);
                    g4r = p_add(ps[0], cb[144 + cul]);
                    g4z = p_add(ps[1], cb[160 + cul]);
                    g4n = p_add(ps[2], cb[176 + cul]);
                }
            }
            RS(10);
            // ---- A6: y3 -> fc4 -> y4 --------------------------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QY3, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(6), (unsigned)t);
            RS(11);
            prod(I1(), 13, cc, PA_F4);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            {
                float y = 0.f;
                if (cell) {
                    float ps[1];
                    psums(I1(), PA_F4, 1, 0, ps);
                    y = p_add(ps[0], cb[208 + cul]);
                    y = y > 0.f ? y : 0.f;
                }
                if (v < 4) pub(QY4, y, seq);
            }
            RS(12);
            // ---- idle while B runs fc5, the sample and GRU1: the partner's ring entry of step
            // t + 3 (its slot (t + 3) & 3 last held step t - 1, whose reads ended in step t - 1).
            // Waves 4-7 never publish, so B's read-after-x2 ordering needs these stores in L2
            // before this half's next publication: drained explicitly here (the
            // wave's next poll would drain them too -- vmcnt counts stores on gfx9 -- but that
            // is a property of the schedule, not of the code), in an idle window.
            ring_make(t + 3);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            RS(13);
        }
        if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[1] = p_now();
        if (ROT && cell && lds[QL_FAIL] == 0.f) {  // the rows' state for their next slice
            int nn = cn;
            asm volatile("" : "+v"(nn));
            float* st = a.st + (size_t)reinterpret_cast<const int2*>(lds + QL_VM)[nn].x * kRRState * RH;
            st[2 * RH + cu] = h2r;
            st[4 * RH + cu] = h4r;
            st[5 * RH + cu] = g2r;
            st[6 * RH + cu] = g2z;
            st[7 * RH + cu] = g2n;
            st[11 * RH + cu] = g4r;
            st[12 * RH + cu] = g4z;
            st[13 * RH + cu] = g4n;
        }
    } else {
        // =============================== half B ===================================
        // slot constants: b_hh1, b_hh3 [3][16], b_f5 [cpw] of the slot's classes
        if (tid < 96) {
            const int gt = (tid % 48) / 16, ul = tid & 15;
            lds[QL_CB + tid] = (tid < 48 ? a.b_hh1 : a.b_hh3)[gt * RH + 16 * s + ul];
        }
        if (tid >= 96 && tid < 96 + a.cpw) {
            const int c = a.cpw * s + tid - 96;
            lds[QL_CB + tid] = c < a.n_classes ? a.b_f5[c] : 0.f;
        }
        float h1r = 0.f, h3r = 0.f, x1c = 0.f;
        float g1r = 0.f, g1z = 0.f, g1n = 0.f, g3r = 0.f, g3z = 0.f, g3n = 0.f;
        if (cell) {  // x1, h1 of step t0 (k_persist_rr_init), h3 = 0: gh3 = b_hh3
            const float* st = a.st + (size_t)crow * kRRState * RH;
            x1c = st[cu];
            h1r = st[RH + cu];
            if (ROT) {  // (a time-sliced row: its chunk state)
                h3r = st[3 * RH + cu];
                g3r = st[8 * RH + cu];
                g3z = st[9 * RH + cu];
                g3n = st[10 * RH + cu];
            } else {
                g3r = a.b_hh3[cu];
                g3z = a.b_hh3[RH + cu];
                g3n = a.b_hh3[2 * RH + cu];
            }
        }
        const float* cb = lds + QL_CB;
        const rsrc_t fcr = mk_rsrc(a.fcond);
        const float vr = cell ? a.v[cu] : 0.f, vz = cell ? a.v[RH + cu] : 0.f, vn = cell ? a.v[2 * RH + cu] : 0.f;
        const float w0c = cell ? a.w0[cu] : 0.f;
        __syncthreads();
        // initial x1, h1 (canonicalised: a signalling NaN in a carried state must not read as
        // the sentinel), as step t0's vectors
        if (v < 4) {
            pub(QX1, __builtin_canonicalizef(x1c), (unsigned)a.t0 + 1u);
            pub(QH1, __builtin_canonicalizef(h1r), (unsigned)a.t0 + 1u);
        }
        for (int t = a.t0; t < a.t1; ++t) {
            const unsigned seq = (unsigned)t + 1u;
            RS(0);
            // per-step cell operands: conditioning of frame(t) (GRU3, fc1, fc3) now; the
            // ring's noise of step t and P1 of step t + 1 (formed by the partner A slot) after
            // the x2 poll below -- A stored them before that publication
            float pc[5] = {0.f, 0.f, 0.f, 0.f, 0.f}, pn[4] = {0.f, 0.f, 0.f, 0.f};
            float4 pp = make_float4(0.f, 0.f, 0.f, 0.f);
            if (cell) {
                const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + QL_RI)[cn];
                const unsigned fo = (unsigned)(p_frame(ri, t, a.hop) * a.cond_width) * 4u;
                int uu = cu;
                asm volatile("" : "+v"(uu));
                pc[0] = bld(fcr, fo + (unsigned)(a.oG3 + uu) * 4u, 0);
                pc[1] = bld(fcr, fo + (unsigned)(a.oG3 + RH + uu) * 4u, 0);
                pc[2] = bld(fcr, fo + (unsigned)(a.oG3 + 2 * RH + uu) * 4u, 0);
                pc[3] = bld(fcr, fo + (unsigned)(a.oF1 + uu) * 4u, 0);
                pc[4] = bld(fcr, fo + (unsigned)(a.oF3 + uu) * 4u, 0);
            }
            // ---- B1: h1 of every B slot -> W_hh1 h1 (GRU1 at this step's end; A runs GRU2) -
            fail |= !q_poll(xr, o_cons, q_slot(QH1, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(7), (unsigned)t);
            RS(1);
            prod(I3(), 0, cc, PB_H1);
            RS(2);
            // ---- B2: x2 -> W_ih3 x2 -> GRU3 -> x3, h3 ---------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QX2, seq), bvalid, o_own, cc, ov, a.ctl, wh(8), (unsigned)t);
            RS(3);
            const float x2v = __uint_as_float(ov);
            if (cell) {  // (non-temporal: the ring lines were written by another CU)
                const unsigned nb = (unsigned)(RG_P + ((t & 3) * kRowsW + cn) * 64 + cul) * 4u;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < ntc) pn[j] = bld_nt(rgr, nb + (unsigned)(16 * j) * 4u, 0);
                pp = bld4_nt(rgr, (unsigned)((((t + 1) & 3) * kRowsW + cn) * 16 + cul) * 16u, 0);
            }
            prod(I3(), 3, cc, PB_G3);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            if (lds[QL_FAIL] != 0.f) return;
            {
                float x3 = 0.f;
                if (cell) {
                    float ps[3];
                    psums(I3(), PB_G3, 3, 0, ps);
                    const float gi0 = p_add(ps[0], pc[0]);
                    const float gi1 = p_add(ps[1], pc[1]);
                    const float gi2 = p_add(ps[2], pc[2]);
                    h3r = p_gru(gi0, gi1, gi2, g3r, g3z, g3n, h3r);
                    x3 = p_add(x2v, h3r);
                }
                if (v < 4) {
                    pub(QX3, x3, seq);
                    pub(QH3, h3r, seq);
                }
                if (cell) {
                    float ps[3];
                    psums(I3(), PB_H1, 3, 0, ps);
                    g1r = p_add(ps[0], cb[cul]);
                    g1z = p_add(ps[1], cb[16 + cul]);
                    g1n = p_add(ps[2], cb[32 + cul]);
                }
            }
            RS(4);
            // ---- B3: h3 of every B slot -> W_hh3 h3 (next step's gh3; A runs GRU4) ----------
            fail |= !q_poll(xr, o_cons, q_slot(QH3, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(9), (unsigned)t);
            prod(I3(), 6, cc, PB_H3);
            RS(5);
            // ---- B4: x4 -> fc1 -> y1 --------------------------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QX4, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(10), (unsigned)t);
            RS(6);
            prod(I1(), 9, cc, PB_F1);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            {
                float y = 0.f;
                if (cell) {
                    float ps[3];
                    psums(I1(), PB_F1, 1, 0, ps);
                    y = p_add(ps[0], pc[3]);
                }
                if (v < 4) pub(QY1, y, seq);
                if (cell) {
                    float ps[3];
                    psums(I3(), PB_H3, 3, 0, ps);
                    g3r = p_add(ps[0], cb[48 + cul]);
                    g3z = p_add(ps[1], cb[64 + cul]);
                    g3n = p_add(ps[2], cb[80 + cul]);
                }
            }
            RS(7);
            // ---- B5: y2 -> fc3 -> y3 --------------------------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QY2, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(11), (unsigned)t);
            RS(8);
            prod(I1(), 10, cc, PB_F3);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            {
                float y = 0.f;
                if (cell) {
                    float ps[1];
                    psums(I1(), PB_F3, 1, 0, ps);
                    y = p_add(ps[0], pc[4]);
                }
                if (v < 4) pub(QY3, y, seq);
            }
            RS(9);
            // ---- B6: y4 -> fc5 -> per-slot candidates ---------------------------------------
            fail |= !q_poll(xr, o_cons, q_slot(QY4, seq), bvalid, o_own_none, cc, ov, a.ctl, wh(12), (unsigned)t);
            RS(10);
            if (ntc == 4)
                prod(std::integral_constant<int, 4>(), 11, cc, PB_F5);
            else
                prod(std::integral_constant<int, 2>(), 11, cc, PB_F5);
            if (fail) lds[QL_FAIL] = 1.f;
            qbar();
            RS(11);
            if (v < 4) {
                const unsigned want = key_tag(seq);
                {
                    // candidate: the max key (cand_key.h cand_key, l_k + G_k formed exactly)
                    // over the slot's classes of row cn: lane cul takes classes cpw s + 16 j + cul,
                    // j < ntc
                    uint32_t kh = 0, kl = 0;
                    if (cell) {
                        float ps[4];
                        if (ntc == 4)
                            psums(I4(), PB_F5, 4, 0, ps);
                        else
                            psums(I2(), PB_F5, 2, 0, ps);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (j >= ntc) break;
                            const int c = a.cpw * s + 16 * j + cul;
                            if (c < a.n_classes) {
                                const float lg = p_add(ps[j], cb[96 + 16 * j + cul]);
                                p_dbg_logit<DBG>(a.dbg, t + roff(cn), crow, c, a.B, a.n_classes, lg);
                                const CandKey k = cand_key(lg, __float_as_uint(pn[j]), c);
                                kmax_take(kh, kl, k.hi, k.lo);
                            }
                        }
                    }
                    row16_kmax(kh, kl);
                    if (cell && cul == 0)
                        __builtin_amdgcn_raw_buffer_store_b64((u2v){kh, kl | want}, xr, q_cand(cn, s), QX_D * 4, 0);
                }
                RS(12);
                // ---- B7: sample of step t (lanes cul < 8 poll slots 2 cul, 2 cul + 1 of row cn)
                float x;
                {
                    u4v q = {0u, want, 0u, want};
                    const unsigned t0s = p_now();
                    unsigned nsp = 0;
                    const bool pl = cell && cul < 8;
                    while (true) {
                        if (pl) {
                            unsigned vo = q_cand(cn, 2 * cul);
                            asm volatile("" : "+v"(vo));
                            q = __builtin_amdgcn_raw_buffer_load_b128(xr, vo, QX_D * 4, kCpNT);
                        }
                        if (__all(((q.y & kKeyTagMask) == want) & ((q.w & kKeyTagMask) == want))) break;
                        if ((++nsp & 63) == 0 && (ld_sc1_u(a.ctl + PC_ERR) || p_now() - t0s > kSpinTicks)) {
                            if (l == 0 && !ld_sc1_u(a.ctl + PC_ERR) &&
                                atomicCAS(a.ctl + PC_WHERE, 0u, wh(13) | ((unsigned)v << 19)) == 0u)
                                a.ctl[PC_WHERE + 2] = (unsigned)t;
                            if (l == 0) atomicMax(a.ctl + PC_ERR, 2u);
                            fail = true;
                            break;
                        }
                    }
                    uint32_t bh = pl ? q.x : 0u, bl = pl ? q.y : 0u;
                    kmax_take(bh, bl, pl ? q.z : 0u, pl ? q.w : 0u);
                    row16_kmax(bh, bl);
                    const int bi = key_cls(bl);
                    {
#pragma clang fp contract(off)
                        x = (2.0f * (float)bi) / (float)(a.n_classes - 1) - 1.0f;
                    }
                    if (s == 0 && cell && cul == 0) {
                        int nn = cn;
                        asm volatile("" : "+v"(nn));
                        unsigned ro = (unsigned)((g0 + kPG * nn) * a.ld);
                        if (ROT) {
                            const int2 vm = reinterpret_cast<const int2*>(lds + QL_VM)[nn];
                            ro = (unsigned)(vm.x * a.ld + vm.y);
                        }
                        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bi, mk_rsrc(a.labels), ro * 2u,
                                                              (unsigned)t * 2u, 0);
                        bst(x, mk_rsrc(a.samples), ro * 4u, (unsigned)t * 4u);
                    }
                }
                if (fail) lds[QL_FAIL] = 1.f;  // seen by every wave at the half's next check
                RS(13);
                // ---- GRU1 of step t + 1 for the slot's units -> x1, h1 ------------------------
                //   gi = W_ih1 (cI + w0 x) + b_ih1 = P1 + v x ; x1 = (cI + w0 x) + h1
                float x1 = 0.f;
                if (cell) {
                    h1r = p_gru(fmaf(vr, x, pp.x), fmaf(vz, x, pp.y), fmaf(vn, x, pp.z), g1r, g1z, g1n, h1r);
                    x1 = p_add(fmaf(w0c, x, pp.w), h1r);
                    if (ROT) x1c = x1;
                }
                pub(QX1, x1, seq + 1u);
                pub(QH1, h1r, seq + 1u);
                RS(14);
            }
            if (s == 0 && tid == 0) {
                if (g == 0) p_progress(a.progress, a.prog_base, t);
                if (p_abort(a.ctl, a.progress, t)) lds[QL_FAIL] = 1.f;  // seen at the half's next check
            }
        }
        if (ROT && cell && lds[QL_FAIL] == 0.f) {  // x1, h1 of step t1 (GRU1 of the last step), h3, gh3
            int nn = cn;
            asm volatile("" : "+v"(nn));
            float* st = a.st + (size_t)reinterpret_cast<const int2*>(lds + QL_VM)[nn].x * kRRState * RH;
            st[cu] = x1c;
            st[RH + cu] = h1r;
            st[3 * RH + cu] = h3r;
            st[8 * RH + cu] = g3r;
            st[9 * RH + cu] = g3z;
            st[10 * RH + cu] = g3n;
        }
    }
#undef QW
#undef RS
}

// launch-side helpers --------------------------------------------------------------------
size_t persist_wide_rr_lds_bytes() { return (size_t)QL_TOTAL * sizeof(float); }
size_t persist_wide_rr_xbuf_floats() { return (size_t)kPG * QX_GROUP; }
size_t persist_wide_rr_ring_floats() { return (size_t)kPG * kHalf * RG_SLOT; }
size_t persist_wide_rr_wreg_floats() { return (size_t)kPM * 8 * kWq * 64 * 4; }
// before every launch: the vector slots to the sentinel, the candidate area (step tags) to 0
__global__ __launch_bounds__(256) void k_wide_rr_xbuf_reset(uint4* x) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)kPG * QX_GROUP / 4) return;
    const unsigned f = (unsigned)((i * 4) % QX_GROUP);
    x[i] = f >= (unsigned)QX_D ? make_uint4(0u, 0u, 0u, 0u) : make_uint4(kSentR, kSentR, kSentR, kSentR);
}
hipError_t persist_wide_rr_reset_xbuf(float* xbuf, hipStream_t s) {
    const unsigned n = (unsigned)((size_t)kPG * QX_GROUP / 4);
    k_wide_rr_xbuf_reset<<<(n + 255) / 256, 256, 0, s>>>(reinterpret_cast<uint4*>(xbuf));
    return hipGetLastError();
}
int persist_wide_rr_scratch() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_persist_wide_rr<false, false>) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}
int persist_wide_rr_rot_scratch() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_persist_wide_rr<true, false>) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}
hipError_t launch_persist_wide_rr(const PersistRRArgs& a, hipStream_t s) {
    // full launches (t0 = 0: the initial state is built in-kernel from k_persist_rr_init's x1,
    // h1) or time-sliced ones (vmap: every row from its chunk state, t1 <= S steps, P1 formed
    // in-kernel), RAW, 512 or 1024 classes (2 or 4 fc5 tiles of 16 per B slot)
    if (a.rb < 0 || a.nr < 1 || a.nr > kPWideRows || a.rb + kPG * a.nr > a.B || a.mode != 0 ||
        a.t0 != 0 || (a.vmap ? a.t1 > a.S || a.p1q == nullptr : a.t1 != a.S) || (a.cpw != 32 && a.cpw != 64) ||
        a.cpw * kHalf < a.n_classes || a.wwide == nullptr || a.wring == nullptr)
        return hipErrorInvalidValue;
    const size_t lb = persist_wide_rr_lds_bytes();
    if (a.vmap) return a.dbg.out ? persist_launch<k_persist_wide_rr<true, true>>(lb, a, s)
                                 : persist_launch<k_persist_wide_rr<true, false>>(lb, a, s);
    return a.dbg.out ? persist_launch<k_persist_wide_rr<false, true>>(lb, a, s)
                     : persist_launch<k_persist_wide_rr<false, false>>(lb, a, s);
}

// Exhaustive host check of the exchange layout (as wide_layout_check for the fatchord kernel):
// for every row count, the producer packets of one hop (16 slots x R rows x 4 unit quads) and
// the consumer packets (8 waves x 64 lanes x 2 packets, lanes of rows >= R off) coincide one to
// one with matching (row, unit quad), inside the slot; a cell's own-value offset lies inside its
// producer's packet; candidates inside their area. Returns the violations.
int wide_rr_layout_check(int R) {
    if (R < 1 || R > kRowsW) return -1;
    int bad = 0;
    std::vector<int> owner(QSLOT / 4, -1);
    for (int s = 0; s < kHalf; ++s)
        for (int cn = 0; cn < R; ++cn)
            for (int cul = 0; cul < 16; cul += 4) {
                const unsigned o = q_prod(s, cn, cul);
                if (o % 16 || o + 16 > (unsigned)QSLOT * 4u) { ++bad; continue; }
                if (owner[o / 16] >= 0) ++bad;
                owner[o / 16] = (s * kRowsW + cn) * 16 + cul;
            }
    int matched = 0;
    for (int v = 0; v < 8; ++v)
        for (int l = 0; l < 64; ++l) {
            if ((l & 15) >= R) continue;
            for (int p = 0; p < 2; ++p) {
                const unsigned o = q_cons(v, l) + 1024u * (unsigned)p;
                if (o % 16 || o + 16 > (unsigned)QSLOT * 4u) { ++bad; continue; }
                const int ow = owner[o / 16];
                if (ow < 0) { ++bad; continue; }
                const int s = ow / (kRowsW * 16), cn = (ow / 16) % kRowsW, cul = ow % 16;
                if (cn != (l & 15) || 16 * s + cul != 32 * v + 8 * (l >> 4) + 4 * p) ++bad;
                ++matched;
            }
        }
    if (matched != kHalf * R * 4) ++bad;
    // a cell's own value (x2 = x1 + h2 etc. read the partner half's x of unit 16 s + cul, row cn):
    // the word o_own = q_prod(s, cn, cul & ~3) + 4 (cul & 3) of the kernel must lie in the packet
    // published for (slot s, row cn, quad cul & ~3), at the word of unit 16 s + cul
    for (int s = 0; s < kHalf; ++s)
        for (int cn = 0; cn < R; ++cn)
            for (int cul = 0; cul < 16; ++cul) {
                const unsigned own = q_prod(s, cn, cul & ~3) + 4u * (unsigned)(cul & 3);
                if (own + 4 > (unsigned)QSLOT * 4u) { ++bad; continue; }
                const int ow = owner[own / 16];
                if (ow != (s * kRowsW + cn) * 16 + (cul & ~3) || (int)((own % 16) / 4) != (cul & 3)) ++bad;
            }
    for (int hb = 0; hb < QN; ++hb)
        for (unsigned sq = 0; sq < 2; ++sq)
            if (q_slot(hb, sq) + (unsigned)QSLOT * 4u > (unsigned)QX_D * 4u ||
                (unsigned long long)kNoOff + q_slot(hb, sq) + 1024ull <= 0x7fffffffull)
                ++bad;
    for (int n = 0; n < R; ++n)
        for (int s = 0; s < kHalf; s += 2)
            if (q_cand(n, s) % 16 || q_cand(n, s) + 16 > (unsigned)(kRowsW * kHalf * 2) * 4u) ++bad;
    return bad;
}

}  // namespace wrnn
