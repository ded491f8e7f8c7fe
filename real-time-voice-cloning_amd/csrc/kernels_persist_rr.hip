// Persistent, weight-stationary recurrence of the runtimeracer WaveRNN (PERSIST engine, second
// topology).
//
// Reference step body: vocoder/models/runtimeracer_version.py:244-270 (rnn_dims = fc_dims = 256):
//   x1 = I(x0) + h1'            h1' = rnn1(I(x0), h1)
//   x2 = x1 + rnn2(x1, h2)      x3 = x2 + rnn3([x2, a2], h3)      x4 = x3 + rnn4(x3, h4)
//   y1 = fc1([x4, a3])          y2 = relu(fc2(y1))
//   y3 = fc3([y2, a4])          y4 = relu(fc4(y3))                 logits = fc5(y4)
//
// Same execution model as kernels_persist.hip: 8 groups of 32 workgroups (one group per XCD,
// formed from HW_REG_XCC_ID), 512 threads per workgroup, every weight of the step resident in
// registers for the whole launch, and in-group exchanges of tagged (value, step) pairs through
// the XCD's shared L2. Slot w owns units / outputs [8w, 8w + 8) of every layer and fc5 classes
// [cpw w, cpw (w + 1)). The 512 threads form four quads of 128 (og = unit 0..7, kc = k-chunk
// 0..15); each quad holds a different set of weight rows (host layout: pack_persist_rr):
//   quad 0: W_ih2 | W_ih3[:, :256] | fc4      quad 1: W_ih4 | W_hh1 | fc3[:, :256]
//   quad 2: W_hh2 | W_hh3 | fc2               quad 3: W_hh4 | fc1[:, :256]
// and in LDS the slot's fc5 rows [32 classes][256] (staged to registers only during stage 8).
// Per step eight hops lie on the dependency chain (GRU2, GRU3, GRU4, fc1, fc2, fc3, fc4, fc5
// candidates) and the recurrent products W_hh h run in the idle quads of earlier stages:
//   stage 1  q0 GRU2 -> (x2, h2)     q1 gh1 = W_hh1 h1 (published)   q3 gh4 = W_hh4 h4 (local)
//   stage 2  q0 GRU3 -> (x3, h3)     q2 gh2 = W_hh2 h2 (next step)
//   stage 3  q1 GRU4 -> (x4, h4)     q2 gh3 = W_hh3 h3 (next step)
//   stage 4  q3 fc1 -> y1            stage 5  q2 fc2 -> y2
//   stage 6  q1 fc3 -> y3            stage 7  q0 fc4 -> y4
//   stage 8  all quads fc5 -> per-slot Gumbel-max candidates (RAW) / logits (MOL)
// then, redundantly in every workgroup, the sample and GRU1 of the next step for all 256 units
// (gi = P1 + v x with P1 = W_ih1 (I c) + b precomputed, the rank-1 x term of kernels_persist.hip).
// Every inter-stage LDS buffer is written only by a poll that follows a barrier after its
// last reader (ping-pong XA / XB for the chain, one buffer per h_k), so no poll races a reader.
#include "wrnn_kernels.h"
#include "persist_common.h"

namespace wrnn {

namespace {

constexpr int RH = kRH;
constexpr int RK4 = RH / 4;    // float4 per row
constexpr int RU = RH / kPM;   // units per slot (8)
static_assert(RU == 8, "quad layout assumes 8 units per slot");

// exchange area per group (floats)
constexpr int RX_G = 0;                                    // GRU hops [3][kRNR][2][RH] pairs
constexpr int RX_G_SZ = kRNR * 2 * RH * 2;
constexpr int RX_F = RX_G + 3 * RX_G_SZ;                   // fc hops [4][kRNR][RH] pairs
constexpr int RX_F_SZ = kRNR * RH * 2;
constexpr int RX_GH1 = RX_F + 4 * RX_F_SZ;                 // gh1 [2 parity][kRNR][RH] (r, z, n, -)
constexpr int RX_GH1_SZ = kRNR * 4 * RH;
constexpr int RX_D = RX_GH1 + 2 * RX_GH1_SZ;               // candidates [kPM][kRNR] pairs
constexpr int RX_D_LOG = kPM * kRNR * 2;
constexpr int RX_GROUP = RX_D + RX_D_LOG + kRNR * 64 + 64; // + MOL logits [kRNR][32] pairs

// LDS carve (floats)
constexpr int L_XA = 0;                          // [kRNR][RH] stage inputs, ping
constexpr int L_XB = L_XA + kRNR * RH;           // pong
constexpr int L_H1 = L_XB + kRNR * RH;           // h1 (W_hh1 input), h2, h3, h4
constexpr int L_H2 = L_H1 + kRNR * RH;
constexpr int L_H3 = L_H2 + kRNR * RH;
constexpr int L_H4 = L_H3 + kRNR * RH;
constexpr int L_GH2 = L_H4 + kRNR * RH;          // [3][RU][kRNR] gh2 = W_hh2 h2 + b (slot units)
constexpr int L_GH3 = L_GH2 + 3 * RU * kRNR;
constexpr int L_GH4 = L_GH3 + 3 * RU * kRNR;
constexpr int L_RED = L_GH4 + 3 * RU * kRNR;     // [32 classes][kRNR][value, class]
constexpr int L_SX = L_RED + 32 * kRNR * 2;      // sampled x per row
constexpr int L_FAIL = L_SX + 8;
constexpr int L_DUMMY = L_SX + 12;               // sink of padding poll lanes (float2)
constexpr int L_RI = L_SX + 16;                  // RowInfo of the group's rows
constexpr int L_VM = L_RI + 6 * kRNR;            // (physical row, step offset) per row slot (rotated)
constexpr int L_CB = L_VM + 2 * kRNR + 4;        // slot constants, see CB_*
constexpr int CB_IH2 = 0, CB_IH4 = 24, CB_HH1 = 48, CB_HH2 = 72, CB_HH3 = 96, CB_HH4 = 120,
              CB_F2 = 144, CB_F4 = 152;
constexpr int L_W5 = L_CB + 160;                 // fc5 rows of the slot [32][RH]
constexpr int L_TOTAL = L_W5 + 32 * RH;
static_assert(L_DUMMY % 2 == 0, "float2 sink");
static_assert(L_W5 % 4 == 0, "float4 weights");

// per-row dot products of register-resident gate rows (3 gates of unit og, k-chunk kc) with the
// NR staged rows of X; lane kc == r of each 16-lane row keeps row r's sums
template <int NR, int B0>
__device__ __forceinline__ void mv3(const float4 (&wr)[kRNW], const float4* X, int kc, float& s0,
                                    float& s1, float& s2) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        v2f acc[3] = {(v2f){0.f, 0.f}, (v2f){0.f, 0.f}, (v2f){0.f, 0.f}};
        float4 xq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) xq[i] = X[r * RK4 + 16 * i + kc];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) dot4(acc[j], wr[B0 + 4 * j + i], xq[i]);
        const float t0 = row16_sum(hsum(acc[0]));
        const float t1 = row16_sum(hsum(acc[1]));
        const float t2 = row16_sum(hsum(acc[2]));
        if (kc == r) {
            s0 = t0;
            s1 = t1;
            s2 = t2;
        }
    }
}
template <int NR, int B0>
__device__ __forceinline__ float mv1(const float4 (&wr)[kRNW], const float4* X, int kc) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        v2f acc = {0.f, 0.f};
        float4 xq[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) xq[i] = X[r * RK4 + 16 * i + kc];
#pragma unroll
        for (int i = 0; i < 4; ++i) dot4(acc, wr[B0 + i], xq[i]);
        const float t = row16_sum(hsum(acc));
        if (kc == r) s = t;
    }
    return s;
}

// Poll one hop of NA arrays x NR rows x RH tagged pairs into LDS (dst0 / dst1 [kRNR][RH]);
// every thread takes couples tid, tid + 512, ...; padding lanes re-poll a valid couple into a
// sink. False on abort / timeout.
// NT threads (tid < NT) poll arrays A0 .. A0 + NA - 1 of a buffer laid out with NL arrays per row
// (GRU hops: NL = 2, x then h); dst0 / dst1 receive the first / second polled array.
template <int NR, int NA, int NT = kPT, int NL = NA, int A0 = 0>
__device__ __forceinline__ bool poll_hop(rsrc_t xr, unsigned so, unsigned seq, float* dst0,
                                         float* dst1, float* sink, unsigned* ctl, int tid) {
    constexpr int TOT = NR * NA * (RH / 2);
    constexpr int M = (TOT + NT - 1) / NT;
    unsigned off[M];
    float2* dst[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int c = tid + NT * m;
        const bool valid = c < TOT;
        const int cc = valid ? c : c % TOT;
        const int r = cc / (NA * (RH / 2)), a = (cc / (RH / 2)) % NA, cp = cc % (RH / 2);
        off[m] = (unsigned)(((r * NL + A0 + a) * RH + 2 * cp) * 8);
        dst[m] = valid ? reinterpret_cast<float2*>((a ? dst1 : dst0) + r * RH) + cp
                       : reinterpret_cast<float2*>(sink);
    }
    return poll_couples<M>(xr, off, so, seq, dst, ctl);
}

// GRU hop carrying h only (X_LOCAL): h -> hdst, and x_next = x_prev + h of the same couples
// (the producer's own fp32 add on the same operands: x_prev is identical in every slot).
template <int NR>
__device__ __forceinline__ bool poll_hop_hx(rsrc_t xr, unsigned so, unsigned seq, float* hdst,
                                            const float* xprev, float* xnext, float* sink,
                                            unsigned* ctl, int tid) {
    constexpr int TOT = NR * (RH / 2);
    constexpr int M = (TOT + kPT - 1) / kPT;
    unsigned off[M];
    float2* dst[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int c = tid + kPT * m;
        const bool valid = c < TOT;
        const int cc = valid ? c : c % TOT;
        const int r = cc / (RH / 2), cp = cc % (RH / 2);
        off[m] = (unsigned)(((r * 2 + 1) * RH + 2 * cp) * 8);
        dst[m] = valid ? reinterpret_cast<float2*>(hdst + r * RH) + cp : reinterpret_cast<float2*>(sink);
    }
    const bool ok = poll_couples<M>(xr, off, so, seq, dst, ctl);
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int c = tid + kPT * m;
        if (c < TOT) {
            const int r = c / (RH / 2), cp = c % (RH / 2);
            const float2 h = *dst[m];
            float2 x = reinterpret_cast<const float2*>(xprev + r * RH)[cp];
            x.x = p_add(x.x, h.x);
            x.y = p_add(x.y, h.y);
            reinterpret_cast<float2*>(xnext + r * RH)[cp] = x;
        }
    }
    return ok;
}

}  // namespace

// DBG: the instance that records logits for the teacher-forced gate (wrnn_set_debug_steps)
// ROT: a rotated launch (PersistRRArgs::vmap, DESIGN.md §3.0e, as kernels_persist.hip): row
//      slot r of the group is the virtual row g + 8 r, mapped to (physical row, step offset);
//      the group runs a.giters[g] steps from its rows' chunk state and saves it at the end; P1
//      and the noise are read at the row's own step, labels / logits written there.
template <int NR, bool MOL, bool ROT, bool DBG>
__device__ __forceinline__ void rr_body(const PersistRRArgs& a, float* lds, const int g, const int w) {
    const int tid = threadIdx.x;
    const int g0 = a.rb + g;                  // first (virtual) fold row of this group in this launch
    const int t1g = ROT ? __builtin_amdgcn_readfirstlane(a.giters[g]) : a.t1;
    auto vmap_g = [&](int r) -> int2 { return ROT ? a.vmap[g0 + kPG * r] : make_int2(g0 + kPG * r, 0); };
    const int q = tid >> 7;                   // quad (wave-uniform)
    const int og = (tid >> 4) & 7, kc = tid & 15;
    const int u = RU * w + og;                // unit / output of this thread's weight rows
    const int cl = 8 * q + og;                // fc5 class of this thread within the slot
    const int cls = a.cpw * w + cl;
    const bool has_cls = cl < a.cpw && cls < a.n_classes;
    const int j = tid & (RH - 1), hs = tid >> 8;  // GRU1: unit j of rows r = 2 i + hs
    constexpr int NRH = (NR + 1) / 2;
    // late h: each GRU hop waits for x only; idle quads fetch h2 / h3 / h4 in the next stage
    // and the off-path W_hh2 h2 / W_hh3 h3 run one stage later (stages 3 / 4)
    constexpr bool HL = true;
    // local x (with late h): the GRU hops carry h only and every slot forms x itself
    // (x1 is identical everywhere: GRU1 runs redundantly), so the late h polls go away
    constexpr bool XL = true;
    const rsrc_t xr = mk_rsrc(a.xbuf + (size_t)g * RX_GROUP);

    // ---- weights -------------------------------------------------------------------------
    float4 wr[kRNW];
    {
        const float4* src = a.wreg + ((size_t)w * kPT + tid) * kRNW;
#pragma unroll
        for (int i = 0; i < kRNW; ++i) wr[i] = src[i];
        const float4* s5 = a.w5 + (size_t)w * 32 * RK4;
        float4* d5 = reinterpret_cast<float4*>(lds + L_W5);
        for (int i = tid; i < 32 * RK4; i += kPT) d5[i] = s5[i];
    }
    // ---- chunk state ----------------------------------------------------------------------
    const size_t SW = (size_t)kRRState * RH;  // state floats per row
    float h1[NRH];
#pragma unroll
    for (int i = 0; i < NRH; ++i) {
        const int r = 2 * i + hs;
        h1[i] = 0.f;
        if (r < NR) {
            const float* st = a.st + (size_t)vmap_g(r).x * SW;
            h1[i] = st[RH + j];
            lds[L_XA + r * RH + j] = st[j];
            lds[L_H1 + r * RH + j] = h1[i];
            lds[L_H4 + r * RH + j] = st[4 * RH + j];
        }
    }
    const bool own = kc < NR;  // lane kc owns (unit u, row kc) in the epilogues
    const int lr = own ? kc : 0;
    const int2 lvm = vmap_g(lr);  // (physical row, step offset) of this lane's epilogue row
    const int lrow = lvm.x;
    float h2r = 0.f, h3r = 0.f, h4r = 0.f;
    if (own) {
        const float* st = a.st + (size_t)lrow * SW;
        if (q == 0) {
            h2r = st[2 * RH + u];
            h3r = st[3 * RH + u];
#pragma unroll
            for (int jg = 0; jg < 3; ++jg) {
                lds[L_GH2 + (jg * RU + og) * kRNR + kc] = st[5 * RH + jg * RH + u];
                lds[L_GH3 + (jg * RU + og) * kRNR + kc] = st[8 * RH + jg * RH + u];
            }
        } else if (q == 1) {
            h4r = st[4 * RH + u];
        }
    }
    if (tid < 24) {
        const int jg = tid >> 3, ul = tid & 7, uu = jg * RH + RU * w + ul;
        lds[L_CB + CB_IH2 + tid] = a.b_ih2[uu];
        lds[L_CB + CB_IH4 + tid] = a.b_ih4[uu];
        lds[L_CB + CB_HH1 + tid] = a.b_hh1[uu];
        lds[L_CB + CB_HH2 + tid] = a.b_hh2[uu];
        lds[L_CB + CB_HH3 + tid] = a.b_hh3[uu];
        lds[L_CB + CB_HH4 + tid] = a.b_hh4[uu];
        if (tid < 8) {
            lds[L_CB + CB_F2 + tid] = a.b_f2[RU * w + tid];
            lds[L_CB + CB_F4 + tid] = a.b_f4[RU * w + tid];
        }
    }
    if (tid < NR) {
        reinterpret_cast<RowInfo*>(lds + L_RI)[tid] = a.rows[g0 + kPG * tid];
        reinterpret_cast<int2*>(lds + L_VM)[tid] = vmap_g(tid);
    }
    if (tid == 0) lds[L_FAIL] = 0.f;
    const float vj0 = a.v[j], vj1 = a.v[RH + j], vj2 = a.v[2 * RH + j], w0j = a.w0[j];
    const float bcls = has_cls ? a.b_f5[cls] : 0.f;
    const rsrc_t fcr = mk_rsrc(a.fcond);
    const unsigned o_tid = (unsigned)j * 4u;
    __syncthreads();

    const float4* XA = reinterpret_cast<const float4*>(lds + L_XA);
    const float4* XB = reinterpret_cast<const float4*>(lds + L_XB);
    float* sink = lds + L_DUMMY;
    const int wave = tid >> 6;
    // GRU hop k (0: x2/h2, 1: x3/h3, 2: x4/h4) pair (row lr, array, unit u); fc hop k pair
    const unsigned o_gx = (unsigned)((lr * 2) * RH + u) * 8u, o_gh = o_gx + RH * 8u;
    const unsigned o_f = (unsigned)(lr * RH + u) * 8u;
    auto sg = [](int k) { return (unsigned)(RX_G + k * RX_G_SZ) * 4u; };
    auto sf = [](int k) { return (unsigned)(RX_F + k * RX_F_SZ) * 4u; };

    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[0] = p_now();
    for (int t = a.t0; t < t1g; ++t) {
        const unsigned seq = (unsigned)t + 1u;
        const bool nxt = t + 1 < a.S;
        const unsigned par = (unsigned)(t & 1);
        // ---- per-step conditioning / noise loads, consumed later in this step ----------------
        float pc0 = 0.f, pc1 = 0.f, pc2 = 0.f;
        if (own) {
            const RowInfo& lri = reinterpret_cast<const RowInfo*>(lds + L_RI)[kc];
            const unsigned fo = (unsigned)(p_frame(lri, t, a.hop) * a.cond_width) * 4u;
            if (q == 0) {  // GRU3: W_ih3[:, 256:] a2 + b_ih3
                const unsigned o = (unsigned)(a.oG3 + u) * 4u + fo;
                pc0 = bld(fcr, o, 0);
                pc1 = bld(fcr, o, RH * 4);
                pc2 = bld(fcr, o, 2 * RH * 4);
            } else if (q == 1) {  // fc3: fc3[:, 256:] a4 + b
                pc0 = bld(fcr, (unsigned)(a.oF3 + u) * 4u + fo, 0);
            } else if (q == 3) {  // fc1: fc1[:, 256:] a3 + b
                pc0 = bld(fcr, (unsigned)(a.oF1 + u) * 4u + fo, 0);
            }
        }
        const float* cb = lds + L_CB;
        // ================= stage 1: q0 GRU2 | q1 gh1 (published) | q3 gh4 (local) ==========
        if (q == 0) {
            __builtin_amdgcn_s_setprio(2);
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 0>(wr, XA, kc, s0, s1, s2);
            if (own) {
                const float* gh = lds + L_GH2 + og * kRNR + kc;
                const float hn = p_gru(p_add(s0, cb[CB_IH2 + og]), p_add(s1, cb[CB_IH2 + 8 + og]),
                                       p_add(s2, cb[CB_IH2 + 16 + og]), gh[0], gh[RU * kRNR],
                                       gh[2 * RU * kRNR], h2r);
                h2r = hn;
                if (!XL) bst_tag(p_add(lds[L_XA + kc * RH + u], hn), seq, xr, o_gx, sg(0));
                bst_tag(hn, seq, xr, o_gh, sg(0));
            }
            __builtin_amdgcn_s_setprio(0);
        } else if (q == 1) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 12>(wr, reinterpret_cast<const float4*>(lds + L_H1), kc, s0, s1, s2);
            if (own) {  // gh1 (r, z, n) of (row kc, unit u): one 16-byte store
                const u4v v = {__float_as_uint(p_add(s0, cb[CB_HH1 + og])),
                               __float_as_uint(p_add(s1, cb[CB_HH1 + 8 + og])),
                               __float_as_uint(p_add(s2, cb[CB_HH1 + 16 + og])), 0u};
                __builtin_amdgcn_raw_buffer_store_b128(
                    v, xr, (unsigned)(((par * kRNR + kc) * RH + u) * 4) * 4u, (unsigned)RX_GH1 * 4u, 0);
            }
            // gh1 reaches L2 before this wave's later publishes (GRU4 at stage 3): a consumer
            // that has seen every slot's x4/h4 tags reads gh1 with plain loads
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (q == 3) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 0>(wr, reinterpret_cast<const float4*>(lds + L_H4), kc, s0, s1, s2);
            if (own) {
                float* gh = lds + L_GH4 + og * kRNR + kc;
                gh[0] = p_add(s0, cb[CB_HH4 + og]);
                gh[RU * kRNR] = p_add(s1, cb[CB_HH4 + 8 + og]);
                gh[2 * RU * kRNR] = p_add(s2, cb[CB_HH4 + 16 + og]);
            }
        }

        if (XL) {
            if (!poll_hop_hx<NR>(xr, sg(0), seq, lds + L_H2, lds + L_XA, lds + L_XB, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        } else if (HL) {
            if (!poll_hop<NR, 1, kPT, 2, 0>(xr, sg(0), seq, lds + L_XB, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        } else {
            if (!poll_hop<NR, 2>(xr, sg(0), seq, lds + L_XB, lds + L_H2, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        }
        __syncthreads();
        // ================= stage 2: q0 GRU3 | q2 gh2 (next step) ============================
        if (q == 0) {
            __builtin_amdgcn_s_setprio(2);
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 12>(wr, XB, kc, s0, s1, s2);
            if (own) {
                const float* gh = lds + L_GH3 + og * kRNR + kc;
                const float hn = p_gru(p_add(s0, pc0), p_add(s1, pc1), p_add(s2, pc2), gh[0],
                                       gh[RU * kRNR], gh[2 * RU * kRNR], h3r);
                h3r = hn;
                if (!XL) bst_tag(p_add(lds[L_XB + kc * RH + u], hn), seq, xr, o_gx, sg(1));
                bst_tag(hn, seq, xr, o_gh, sg(1));
            }
            __builtin_amdgcn_s_setprio(0);
        } else if (q == 2 && !HL) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 0>(wr, reinterpret_cast<const float4*>(lds + L_H2), kc, s0, s1, s2);
            if (own) {
                float* gh = lds + L_GH2 + og * kRNR + kc;
                gh[0] = p_add(s0, cb[CB_HH2 + og]);
                gh[RU * kRNR] = p_add(s1, cb[CB_HH2 + 8 + og]);
                gh[2 * RU * kRNR] = p_add(s2, cb[CB_HH2 + 16 + og]);
            }
        } else if ((q & 1) && HL && !XL) {  // q1, q3: h2 of every slot (published with x2 at stage 1)
            if (!poll_hop<NR, 1, 256, 2, 1>(xr, sg(0), seq, lds + L_H2, nullptr, sink, a.ctl,
                                            ((q >> 1) << 7) | (tid & 127)))
                lds[L_FAIL] = 1.f;
        }
        if (XL) {
            if (!poll_hop_hx<NR>(xr, sg(1), seq, lds + L_H3, lds + L_XB, lds + L_XA, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        } else if (HL) {
            if (!poll_hop<NR, 1, kPT, 2, 0>(xr, sg(1), seq, lds + L_XA, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        } else {
            if (!poll_hop<NR, 2>(xr, sg(1), seq, lds + L_XA, lds + L_H3, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        }
        __syncthreads();
        // ================= stage 3: q1 GRU4 | q2 gh3 (next step) ============================
        if (q == 1) {
            __builtin_amdgcn_s_setprio(2);
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 0>(wr, XA, kc, s0, s1, s2);
            if (own) {
                const float* gh = lds + L_GH4 + og * kRNR + kc;
                const float hn = p_gru(p_add(s0, cb[CB_IH4 + og]), p_add(s1, cb[CB_IH4 + 8 + og]),
                                       p_add(s2, cb[CB_IH4 + 16 + og]), gh[0], gh[RU * kRNR],
                                       gh[2 * RU * kRNR], h4r);
                h4r = hn;
                if (!XL) bst_tag(p_add(lds[L_XA + kc * RH + u], hn), seq, xr, o_gx, sg(2));
                bst_tag(hn, seq, xr, o_gh, sg(2));
            }
            __builtin_amdgcn_s_setprio(0);
        } else if (q == 2) {  // H_LATE: gh2 here (h2 staged in stage 2), gh3 in stage 4
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            if (HL)
                mv3<NR, 0>(wr, reinterpret_cast<const float4*>(lds + L_H2), kc, s0, s1, s2);
            else
                mv3<NR, 12>(wr, reinterpret_cast<const float4*>(lds + L_H3), kc, s0, s1, s2);
            if (own) {
                const int ob = HL ? CB_HH2 : CB_HH3;
                float* gh = lds + (HL ? L_GH2 : L_GH3) + og * kRNR + kc;
                gh[0] = p_add(s0, cb[ob + og]);
                gh[RU * kRNR] = p_add(s1, cb[ob + 8 + og]);
                gh[2 * RU * kRNR] = p_add(s2, cb[ob + 16 + og]);
            }
        } else if ((q == 0 || q == 3) && HL && !XL) {  // h3 of every slot (published with x3 at stage 2)
            if (!poll_hop<NR, 1, 256, 2, 1>(xr, sg(1), seq, lds + L_H3, nullptr, sink, a.ctl,
                                            ((q & 1) << 7) | (tid & 127)))
                lds[L_FAIL] = 1.f;
        }
        if (XL) {
            if (!poll_hop_hx<NR>(xr, sg(2), seq, lds + L_H4, lds + L_XA, lds + L_XB, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        } else if (HL) {
            if (!poll_hop<NR, 1, kPT, 2, 0>(xr, sg(2), seq, lds + L_XB, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        } else {
            if (!poll_hop<NR, 2>(xr, sg(2), seq, lds + L_XB, lds + L_H4, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        }
        __syncthreads();
        // GRU1 operands of the end of this step: every slot's gh1 is in L2 (drained before its
        // x4/h4 publish, all of which this workgroup has seen)
        float pG[NRH][3];
#pragma unroll
        for (int i = 0; i < NRH; ++i) {
            const int r = 2 * i + hs < NR ? 2 * i + hs : 0;
            const u4v v = __builtin_amdgcn_raw_buffer_load_b128(
                xr, o_tid * 4u, (unsigned)(RX_GH1 + (par * kRNR + r) * 4 * RH) * 4u, kCpNT);
            pG[i][0] = __uint_as_float(v.x);
            pG[i][1] = __uint_as_float(v.y);
            pG[i][2] = __uint_as_float(v.z);
        }
        // P1 / cI of step t+1 for the same GRU1 (HBM latency hides behind stages 4-8)
        float pP[NRH][3], pC[NRH];
        {  // (unconditional, step clamped: every path to the back edge consumes these loads)
            const int tn = nxt ? t + 1 : t;
            // P1 is [step][row][unit][r, z, n, cI]: one 16-byte load per row
            const rsrc_t pr = mk_rsrc(a.P1 + ((size_t)tn * a.B + g0) * 4 * RH);
#pragma unroll
            for (int i = 0; i < NRH; ++i) {
                const int r = 2 * i + hs;
                if (r < NR) {
                    u4v v;
                    if constexpr (ROT) {  // row r (wave-uniform) at its own step, clamped to S - 1
                        const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[r];
                        const int px = __builtin_amdgcn_readfirstlane(vm.x), po = __builtin_amdgcn_readfirstlane(vm.y);
                        const int ts = t + 1 + po < a.S ? t + 1 + po : a.S - 1;
                        v = __builtin_amdgcn_raw_buffer_load_b128(
                            mk_rsrc(a.P1 + ((size_t)ts * a.B + px) * 4 * RH), o_tid * 4u, 0, 0);
                    } else {
                        v = __builtin_amdgcn_raw_buffer_load_b128(pr, o_tid * 4u, (unsigned)(r * kPG * 4 * RH) * 4u, 0);
                    }
                    pP[i][0] = __uint_as_float(v.x);
                    pP[i][1] = __uint_as_float(v.y);
                    pP[i][2] = __uint_as_float(v.z);
                    pC[i] = __uint_as_float(v.w);
                }
            }
        }
        float pgum = 0.f;  // Gumbel noise of (row kc, class cls), step t
        if (own && has_cls && !MOL) {
            if constexpr (ROT)  // (the row's own step; the stream < 4 GiB, runtime-checked)
                pgum = bld(mk_rsrc(a.gumbel),
                           (unsigned)((((unsigned)(t + lvm.y) * (unsigned)a.B + (unsigned)lrow) * (unsigned)a.n_classes +
                                       (unsigned)cls) * 4u), 0);
            else
                pgum = bld(mk_rsrc(a.gumbel + (size_t)t * a.B * a.n_classes),
                           (unsigned)(lrow * a.n_classes + cls) * 4u, 0);
        }
        // MOL: sampling lane (row tid / 32, k = tid % 32 < 11) holds draw k of its row
        if (MOL && tid < 32 * NR && (tid & 31) < 11) {
            size_t ro = (size_t)t * a.B + g0 + kPG * (tid >> 5);
            if constexpr (ROT) {  // (the row's own step)
                const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[tid >> 5];
                ro = (size_t)(t + vm.y) * a.B + vm.x;
            }
            pgum = bld(mk_rsrc(a.gumbel + ro * kMolNoise), (unsigned)(tid & 31) * 4u, 0);
        }
        // ================= stage 4: q3 fc1 ==================================================
        if (q == 3) {
            __builtin_amdgcn_s_setprio(2);
            const float s = mv1<NR, 12>(wr, XB, kc);
            if (own) bst_tag(p_add(s, pc0), seq, xr, o_f, sf(0));
            __builtin_amdgcn_s_setprio(0);
        } else if (q == 2 && HL) {  // gh3 = W_hh3 h3 + b (next step's GRU3; h3 staged in stage 3)
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3<NR, 12>(wr, reinterpret_cast<const float4*>(lds + L_H3), kc, s0, s1, s2);
            if (own) {
                float* gh = lds + L_GH3 + og * kRNR + kc;
                gh[0] = p_add(s0, cb[CB_HH3 + og]);
                gh[RU * kRNR] = p_add(s1, cb[CB_HH3 + 8 + og]);
                gh[2 * RU * kRNR] = p_add(s2, cb[CB_HH3 + 16 + og]);
            }
        }
        if (!poll_hop<NR, 1>(xr, sf(0), seq, lds + L_XA, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        __syncthreads();
        // ================= stage 5: q2 fc2 (relu) ===========================================
        if (q == 2) {
            __builtin_amdgcn_s_setprio(2);
            const float s = mv1<NR, 24>(wr, XA, kc);
            if (own) {
                const float y = p_add(s, cb[CB_F2 + og]);
                bst_tag(y > 0.f ? y : 0.f, seq, xr, o_f, sf(1));
            }
            __builtin_amdgcn_s_setprio(0);
        } else if ((q & 1) && HL && !XL) {  // q1, q3: h4 of every slot (published with x4 at stage 3;
                                     // their GRU1 loads have landed: the hop-4 poll waited on them)
            if (!poll_hop<NR, 1, 256, 2, 1>(xr, sg(2), seq, lds + L_H4, nullptr, sink, a.ctl,
                                            ((q >> 1) << 7) | (tid & 127)))
                lds[L_FAIL] = 1.f;
        }
        if (!poll_hop<NR, 1>(xr, sf(1), seq, lds + L_XB, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        __syncthreads();
        // ================= stage 6: q1 fc3 ==================================================
        if (q == 1) {
            __builtin_amdgcn_s_setprio(2);
            const float s = mv1<NR, 24>(wr, XB, kc);
            if (own) bst_tag(p_add(s, pc0), seq, xr, o_f, sf(2));
            __builtin_amdgcn_s_setprio(0);
        }
        if (!poll_hop<NR, 1>(xr, sf(2), seq, lds + L_XA, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        __syncthreads();
        // ================= stage 7: q0 fc4 (relu) ===========================================
        if (q == 0) {
            __builtin_amdgcn_s_setprio(2);
            const float s = mv1<NR, 24>(wr, XA, kc);
            if (own) {
                const float y = p_add(s, cb[CB_F4 + og]);
                bst_tag(y > 0.f ? y : 0.f, seq, xr, o_f, sf(3));
            }
            __builtin_amdgcn_s_setprio(0);
        }
        if (!poll_hop<NR, 1>(xr, sf(3), seq, lds + L_XB, nullptr, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        __syncthreads();
        // ================= stage 8: fc5 -> per-slot candidates (RAW) / logits (MOL) =========
        {
            float s0 = 0.f;
            if (8 * q < a.cpw) {  // wave-uniform skip of idle quads
                const float4* W5 = reinterpret_cast<const float4*>(lds + L_W5) + cl * RK4;
                float4 w5[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) w5[i] = W5[16 * i + kc];
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    v2f acc = {0.f, 0.f};
#pragma unroll
                    for (int i = 0; i < 4; ++i) dot4(acc, w5[i], XB[r * RK4 + 16 * i + kc]);
                    const float tt = row16_sum(hsum(acc));
                    if (kc == r) s0 = tt;
                }
            }
            // [cl][r] (logit, noise word): wave 0 forms the candidate keys (cand_key) as it
            // reduces them; MOL: the logit, published after the barrier below
            float* red = lds + L_RED;
            if (own) {
                float l = -INFINITY;
                if (has_cls) {
                    l = p_add(s0, bcls);
                    p_dbg_logit<DBG>(a.dbg, t + (ROT ? lvm.y : 0), lrow, cls, a.B, a.n_classes, l);
                }
                *reinterpret_cast<float2*>(red + (cl * kRNR + kc) * 2) = make_float2(l, pgum);
            }
            __syncthreads();
            if (wave == 0) {
                if (!MOL) {
                    // slot candidate per row: the max key, tagged with the step
                    const unsigned tag = key_tag(seq);
                    if (a.cpw <= 16) {  // DPP row r = lane / 16 reduces the slot's classes of row r
                        const int r = tid >> 4, o = tid & 15;
                        uint32_t bh = 0, bl = 0;
                        if (r < NR && o < a.cpw && a.cpw * w + o < a.n_classes) {
                            const float2 lg = *reinterpret_cast<const float2*>(red + (o * kRNR + r) * 2);
                            const CandKey k = cand_key(lg.x, __float_as_uint(lg.y), a.cpw * w + o);
                            bh = k.hi;
                            bl = k.lo;
                        }
                        row16_kmax(bh, bl);
                        if (r < NR && o == 0)
                            __builtin_amdgcn_raw_buffer_store_b64((u2v){bh, bl | tag}, xr,
                                                                  (unsigned)((w * kRNR + r) * 2) * 4u, RX_D * 4, 0);
                    } else {
#pragma unroll
                        for (int rb = 0; rb < NR; rb += 2) {
                            const int r = rb + (tid >> 5), o = tid & 31;
                            uint32_t bh = 0, bl = 0;
                            if (r < NR && o < a.cpw && a.cpw * w + o < a.n_classes) {
                                const float2 lg = *reinterpret_cast<const float2*>(red + (o * kRNR + r) * 2);
                                const CandKey k = cand_key(lg.x, __float_as_uint(lg.y), a.cpw * w + o);
                                bh = k.hi;
                                bl = k.lo;
                            }
                            half_kmax(bh, bl);
                            if (r < NR && o == 31)
                                __builtin_amdgcn_raw_buffer_store_b64((u2v){bh, bl | tag}, xr,
                                                                      (unsigned)((w * kRNR + r) * 2) * 4u, RX_D * 4, 0);
                        }
                    }
                } else {
                    // MOL: the slot's logits (row r, class c) as tagged pairs, polled directly
                    // by every workgroup's sampling lanes
                    const int r = tid >> 4, c = tid & 15;
                    if (r < NR && c < a.cpw && a.cpw * w + c < a.n_classes)
                        bst_tag(red[(c * kRNR + r) * 2], seq, xr, (unsigned)(r * 32 + a.cpw * w + c) * 8u,
                                (RX_D + RX_D_LOG) * 4);
                }
            }
        }
        // ================= sample of step t (redundant in every workgroup) ==================
        if (!MOL) {
            if (tid < 32 * NR) {  // half-wave r: lane o polls slot o's tagged candidate of row r
                const int r = tid >> 5, o = tid & 31;
                const unsigned off = (unsigned)((o * kRNR + r) * 2) * 4u;
                const unsigned want = key_tag(seq);
                u2v c;
                const unsigned ts = p_now();
                unsigned n = 0;
                while (true) {
                    c = __builtin_amdgcn_raw_buffer_load_b64(xr, off, RX_D * 4, kCpNT);
                    if (__all((c.y & kKeyTagMask) == want)) break;
                    if ((++n & 255) == 0) {
                        if (ld_sc1_u(a.ctl + PC_ERR) || p_now() - ts > kSpinTicks) {
                            if ((tid & 63) == 0) atomicMax(a.ctl + PC_ERR, 2u);
                            lds[L_FAIL] = 1.f;
                            break;
                        }
                    }
                }
                uint32_t bh = c.x, bl = c.y;
                half_kmax(bh, bl);  // the 32 slots' candidates: argmax over all classes of row r
                if (o == 31) {
                    const int bi = key_cls(bl);
                    float xv;
                    {
#pragma clang fp contract(off)
                        xv = (2.0f * (float)bi) / (float)(a.n_classes - 1) - 1.0f;
                    }
                    lds[L_SX + r] = xv;
                    if (w == 0) {
                        unsigned ro = (unsigned)((g0 + kPG * r) * a.ld);
                        if (ROT) {
                            const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[r];
                            ro = (unsigned)(vm.x * a.ld + vm.y);
                        }
                        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bi, mk_rsrc(a.labels),
                                                              ro * 2u, (unsigned)t * 2u, 0);
                        bst(xv, mk_rsrc(a.samples), ro * 4u, (unsigned)t * 4u);
                    }
                }
            }
        } else if (tid < 32 * NR) {
            // MOL: vocoder/distribution.py:104-140. Half-wave r: lane k polls logit k of row r
            // (tagged pair) and holds draw k of k_mol_noise (gm_k = log(-log(u1_k)), k < 10;
            // gm_10 = log(u2) - log(1 - u2))
            const int r = tid >> 5, k = tid & 31, row = g0 + kPG * r;
            const unsigned so = (RX_D + RX_D_LOG) * 4;
            const unsigned off = (unsigned)(r * 32 + k) * 8u;
            const bool real = k < a.n_classes;
            const unsigned ts = p_now();
            unsigned n = 0;
            u2v c = __builtin_amdgcn_raw_buffer_load_b64(xr, off, so, kCpNT);
            while (true) {  // two polls in flight
                const u2v c1 = __builtin_amdgcn_raw_buffer_load_b64(xr, off, so, kCpNT);
                if (__all(!real || c.y == seq)) break;
                c = c1;
                if ((++n & 255) == 0) {
                    if (ld_sc1_u(a.ctl + PC_ERR) || p_now() - ts > kSpinTicks) {
                        if ((tid & 63) == 0) atomicMax(a.ctl + PC_ERR, 2u);
                        lds[L_FAIL] = 1.f;
                        break;
                    }
                }
            }
            const float lk = __uint_as_float(c.x);
            const int base = (tid & 63) & 32;
            float bv;
            {
#pragma clang fp contract(off)
                bv = k < 10 ? lk - pgum : -INFINITY;
            }
            int bi = k < 10 ? k : 0x7fffffff;
            row16_argmax(bv, bi);  // first max over k < 10
            bi = __shfl(bi, base);
            bi = bi < 10 ? bi : 0;
            const float mean = __shfl(lk, base + 10 + bi);
            float ls = __shfl(lk, base + 20 + bi);
            const float lu = __shfl(pgum, base + 10);
            if (k == 0) {
                float xv;
                {
#pragma clang fp contract(off)
                    const float lsmin = -32.23619130191664f;  // float(np.log(1e-14))
                    ls = ls < lsmin ? lsmin : ls;
                    xv = mean + expf(ls) * lu;
                    xv = xv < -1.f ? -1.f : xv;
                    xv = xv > 1.f ? 1.f : xv;
                }
                lds[L_SX + r] = xv;
                if (w == 0) {
                    unsigned ro = (unsigned)(row * a.ld);
                    if (ROT) {
                        const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[r];
                        ro = (unsigned)(vm.x * a.ld + vm.y);
                    }
                    bst(xv, mk_rsrc(a.samples), ro * 4u, (unsigned)t * 4u);
                }
            }
        }
        __syncthreads();
        // the step's one failure check (as kernels_persist.hip): a wave whose poll gave up
        // finishes the step, every other poll of it ends within a few spins of PC_ERR
        if (lds[L_FAIL] != 0.f) return;
        // (at the last step this GRU1 runs on clamped inputs and its result goes unused)
        // ================= GRU1 of step t+1 for all 256 units (redundant) ===================
#pragma unroll
        for (int i = 0; i < NRH; ++i) {
            const int r = 2 * i + hs;
            if (r < NR) {
                const float x = lds[L_SX + r];
                const float hn = p_gru(fmaf(vj0, x, pP[i][0]), fmaf(vj1, x, pP[i][1]),
                                       fmaf(vj2, x, pP[i][2]), pG[i][0], pG[i][1], pG[i][2], h1[i]);
                h1[i] = hn;
                lds[L_XA + r * RH + j] = p_add(fmaf(w0j, x, pC[i]), hn);
                lds[L_H1 + r * RH + j] = hn;
            }
        }
        if (w == 0 && tid == 0) {
            // (rotated: the launch's share of the call, steps scaled to S per launch)
            if (g == 0) p_progress(a.progress, a.prog_base, ROT ? (int)((long long)t * a.S / t1g) : t, t);
            if (p_abort(a.ctl, a.progress, t)) lds[L_FAIL] = 1.f;  // seen at the next step's check
        }
        __syncthreads();
    }
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[1] = p_now();
    // ---- save the chunk state ----------------------------------------------------------------
    // (lane indices recomputed here: values kept alive across the step loop cost registers)
    if (ROT || a.t1 < a.S) {
        int tx = tid;
        asm volatile("" : "+v"(tx));
        const int jx = tx & (RH - 1), hx = tx >> 8, kx = tx & 15;
        const int ux = RU * w + ((tx >> 4) & 7), rx = vmap_g(kx < NR ? kx : 0).x;
        if (w == 0)
#pragma unroll
            for (int i = 0; i < NRH; ++i) {
                const int r = 2 * i + hx;
                if (r < NR) {
                    float* st = a.st + (size_t)vmap_g(r).x * SW;
                    st[jx] = lds[L_XA + r * RH + jx];
                    st[RH + jx] = lds[L_H1 + r * RH + jx];
                }
            }
        if (own) {
            float* st = a.st + (size_t)rx * SW;
            if (q == 0) {
                st[2 * RH + ux] = h2r;
                st[3 * RH + ux] = h3r;
#pragma unroll
                for (int jg = 0; jg < 3; ++jg) {
                    st[5 * RH + jg * RH + ux] = lds[L_GH2 + (jg * RU + og) * kRNR + kc];
                    st[8 * RH + jg * RH + ux] = lds[L_GH3 + (jg * RU + og) * kRNR + kc];
                }
            } else if (q == 1) {
                st[4 * RH + ux] = h4r;
            }
        }
    }
}

template <int NR, bool MOL, bool ROT, bool DBG>
__global__ __launch_bounds__(kPT, 1) void k_persist_rr(PersistRRArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_group, s_slot, s_ok;
    // ---- group formation (as kernels_persist.hip) -------------------------------------------
    if (threadIdx.x == 0) {
        int gg, ss;
        s_ok = p_register(a.ctl, gg, ss);
        s_group = gg;
        s_slot = ss;
    }
    __syncthreads();
    if (!s_ok) return;
    const int g = __builtin_amdgcn_readfirstlane(s_group);
    const int w = __builtin_amdgcn_readfirstlane(s_slot);
    if constexpr (ROT && NR >= 2) {  // each group runs its own row count's body
        if (__builtin_amdgcn_readfirstlane(a.gnr[g]) == NR)
            rr_body<NR, MOL, true, DBG>(a, lds, g, w);
        else
            rr_body<NR - 1, MOL, true, DBG>(a, lds, g, w);
    } else {
        rr_body<NR, MOL, false, DBG>(a, lds, g, w);
    }
}

// Step-0 state: GRU1 with x = 0, h = 0 (gh = b_hh1) -> x1(0), h1(0); h2 = h3 = h4 = 0,
// gh2 = b_hh2, gh3 = b_hh3, gh4 = b_hh4.
__global__ __launch_bounds__(kRH) void k_persist_rr_init(PersistRRArgs a) {
    const int row = blockIdx.x, j = threadIdx.x, H = kRH;
    const float* P1 = a.P1 + ((size_t)row * H + j) * 4;  // step 0: (r, z, n, cI) of unit j
    const float hn = p_gru(P1[0], P1[1], P1[2], a.b_hh1[j], a.b_hh1[H + j],
                           a.b_hh1[2 * H + j], 0.f);
    float* st = a.st + (size_t)row * kRRState * H;
    st[j] = p_add(P1[3], hn);
    st[H + j] = hn;
    st[2 * H + j] = 0.f;
    st[3 * H + j] = 0.f;
    st[4 * H + j] = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        st[5 * H + k * H + j] = a.b_hh2[k * H + j];
        st[8 * H + k * H + j] = a.b_hh3[k * H + j];
        st[11 * H + k * H + j] = a.b_hh4[k * H + j];
    }
}

hipError_t launch_persist_rr_init(const PersistRRArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_persist_rr_init, dim3(a.B), dim3(kRH), 0, s, a);
    return hipGetLastError();
}

size_t persist_rr_lds_bytes() { return (size_t)L_TOTAL * sizeof(float); }
size_t persist_rr_xbuf_floats() { return (size_t)kPG * RX_GROUP; }

template <int NR, bool MOL>
hipError_t launch_persist_rr_t(const PersistRRArgs& a, hipStream_t s) {
    if constexpr (NR >= 2) {
        if (a.vmap) {  // rotated (RAW / MOL, 2-4 rows per group)
            if (a.dbg.out) return persist_launch<k_persist_rr<NR, MOL, true, true>>(persist_rr_lds_bytes(), a, s);
            return persist_launch<k_persist_rr<NR, MOL, true, false>>(persist_rr_lds_bytes(), a, s);
        }
    }
    if (a.vmap) return hipErrorInvalidValue;
    if (a.dbg.out) return persist_launch<k_persist_rr<NR, MOL, false, true>>(persist_rr_lds_bytes(), a, s);
    return persist_launch<k_persist_rr<NR, MOL, false, false>>(persist_rr_lds_bytes(), a, s);
}

template <int NR, bool MOL>
int persist_rr_spill_t() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_persist_rr<NR, MOL, false, false>) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}
// scratch bytes of the rotated RAW / MOL instance of nr (2-4) rows per group; -1 if none
int persist_rr_rot_scratch(int nr, bool mol) {
    hipFuncAttributes fa;
    const void* f = nullptr;
    if (!mol)
        f = nr == 2 ? (const void*)k_persist_rr<2, false, true, false>
          : nr == 3 ? (const void*)k_persist_rr<3, false, true, false>
          : nr == 4 ? (const void*)k_persist_rr<4, false, true, false> : nullptr;
    else
        f = nr == 2 ? (const void*)k_persist_rr<2, true, true, false>
          : nr == 3 ? (const void*)k_persist_rr<3, true, true, false>
          : nr == 4 ? (const void*)k_persist_rr<4, true, true, false> : nullptr;
    if (!f || hipFuncGetAttributes(&fa, f) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}

template <bool MOL>
int persist_rr_spill_nr(int nr) {
    switch (nr) {
        case 1: return persist_rr_spill_t<1, MOL>();
        case 2: return persist_rr_spill_t<2, MOL>();
        case 3: return persist_rr_spill_t<3, MOL>();
        case 4: return persist_rr_spill_t<4, MOL>();
        default: return -1;
    }
}

int persist_rr_variant_ok(int nr, int cpw, int mode) {
    if (cpw < 1 || cpw > 32 || (mode != 0 && cpw > 16)) return 0;
    const int sp = mode != 0 ? persist_rr_spill_nr<true>(nr) : persist_rr_spill_nr<false>(nr);
    return sp == 0 ? 1 : 0;
}

template <bool MOL>
hipError_t launch_persist_rr_m(const PersistRRArgs& a, hipStream_t s) {
    switch (a.nr) {
        case 1: return launch_persist_rr_t<1, MOL>(a, s);
        case 2: return launch_persist_rr_t<2, MOL>(a, s);
        case 3: return launch_persist_rr_t<3, MOL>(a, s);
        case 4: return launch_persist_rr_t<4, MOL>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_persist_rr(const PersistRRArgs& a, hipStream_t s) {
    if (a.rb < 0 || a.nr < 1 || a.rb + kPG * a.nr > a.B || a.cpw < 1 || a.cpw > 32 ||
        a.cpw * kPM < a.n_classes || (a.mode != 0 && (a.n_classes > 32 || a.cpw > 16)))
        return hipErrorInvalidValue;
    return a.mode != 0 ? launch_persist_rr_m<true>(a, s) : launch_persist_rr_m<false>(a, s);
}

}  // namespace wrnn
