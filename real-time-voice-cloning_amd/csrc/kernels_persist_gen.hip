// Persistent, weight-stationary recurrence of the geneing WaveRNN (PERSIST engine, third
// topology).
//
// Reference step body: vocoder/models/geneing_version.py:193-205 (rnn_dims 256, fc_dims 128):
//   x1 = I(x0) + h1'     h1' = rnn1(I(x0), h1)
//   y1 = relu(fc1([x1, a2]))        logits = fc3(y1)
//
// Execution model of kernels_persist.hip / kernels_persist_rr.hip: 8 XCD-local groups of 32
// workgroups x 512 threads, all step weights register-resident, tagged (value, step) pairs
// exchanged through the XCD's L2. Slot w owns GRU units [8w, 8w + 8), fc1 outputs
// [4w, 4w + 4) and fc3 classes [cpw w, cpw (w + 1)). Threads form four quads of 128
// (og = 0..7, kc = k-chunk 0..15); host layout (pack_persist_gen):
//   quad 0: W_hh1 rows of unit 8 w + og (3 gates x 4 float4)   @0
//   quad 1: fc1[:, :256] row 4 w + og, og < 4 (4 float4)        @0
//   every quad: fc3 row of class cpw w + 8 q + og (K = 128: 2 float4) @12
// Per step, two hops lie on the dependency chain:
//   stage 1  q1 fc1 -> y1 (hop 1)        q0 gh1 = W_hh1 h1 + b (tagged pairs, read in stage 2)
//   stage 2  fc3 over all quads -> per-slot Gumbel-max candidates (hop 2) / MOL logits;
//            every thread also polls this step's gh1 pairs into LDS before the candidates are
//            published (so no producer can overwrite them first)
// then, redundantly in every workgroup, the sample and GRU1 of the next step (rank-1 x term).
#include "wrnn_kernels.h"
#include "persist_common.h"
#include "philox.h"

namespace wrnn {

namespace {

constexpr int GH = 256;        // rnn_dims
constexpr int GK4 = GH / 4;
constexpr int GF = kGF;        // fc_dims
constexpr int GFK4 = GF / 4;
constexpr int GU = GH / kPM;   // GRU units per slot (8)
constexpr int GO = GF / kPM;   // fc1 outputs per slot (4)
constexpr int GNR = kRNR;      // max rows per group (4)

// exchange area per group (floats)
constexpr int QX_Y = 0;                                  // fc1 hop [GNR][GF] pairs
constexpr int QX_GH = QX_Y + GNR * GF * 2;               // gh1 [GNR][3 GH] pairs
constexpr int QX_D = QX_GH + GNR * 3 * GH * 2;           // candidates [kPM][GNR] pairs
constexpr int QX_D_LOG = kPM * GNR * 2;
constexpr int QX_GROUP = QX_D + QX_D_LOG + GNR * 64 + 64;  // + MOL / BETA logits [GNR][32] pairs

// LDS carve (floats)
constexpr int L_XA = 0;                        // [GNR][GH] x1 (fc1 input)
constexpr int L_H1 = L_XA + GNR * GH;          // [GNR][GH] h1 (W_hh1 input)
constexpr int L_Y = L_H1 + GNR * GH;           // [GNR][GF] y1 (fc3 input)
constexpr int L_GH = L_Y + GNR * GF;           // [GNR][3 GH] gh1 of this step (polled)
constexpr int L_RED = L_GH + GNR * 3 * GH;     // [32][GNR][value, class]
constexpr int L_SX = L_RED + 32 * GNR * 2;
constexpr int L_FAIL = L_SX + 8;
constexpr int L_DUMMY = L_SX + 12;
constexpr int L_RI = L_SX + 16;
constexpr int L_VM = L_RI + 6 * GNR + 4;       // (physical row, step offset) per row slot (rotated)
constexpr int L_CB = L_VM + 2 * GNR + 4;       // b_hh1 of the slot's units [3][8]
constexpr int L_TOTAL = L_CB + 24;
static_assert(L_DUMMY % 2 == 0 && L_VM % 2 == 0, "float2 sink, int2 row map");

// poll NPAIR tagged pairs per row x NR rows into LDS dst[r * NPAIR + ...]
template <int NR, int NPAIR>
__device__ __forceinline__ bool poll_rows(rsrc_t xr, unsigned so, unsigned seq, float* dst, float* sink,
                                          unsigned* ctl, int tid) {
    constexpr int CPR = NPAIR / 2;  // couples per row
    constexpr int TOT = NR * CPR;
    constexpr int M = (TOT + kPT - 1) / kPT;
    unsigned off[M];
    float2* d[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int c = tid + kPT * m;
        const bool valid = c < TOT;
        const int cc = valid ? c : c % TOT;
        const int r = cc / CPR, cp = cc % CPR;
        off[m] = (unsigned)((r * NPAIR + 2 * cp) * 8);
        d[m] = valid ? reinterpret_cast<float2*>(dst + r * NPAIR) + cp : reinterpret_cast<float2*>(sink);
    }
    return poll_couples<M, true>(xr, off, so, seq, d, ctl);  // first pass loads every couple
}

}  // namespace

// MODE: 0 RAW (categorical, 'BITS'), 1 MOL, 2 BETA (geneing 'RAW'); each its own instantiation
// DBG: the instance that records logits for the teacher-forced gate (wrnn_set_debug_steps)
// ROT: a rotated launch (PersistGenArgs::vmap, DESIGN.md §3.0e, as kernels_persist_rr.hip): row
//      slot r of the group is the virtual row g + 8 r, mapped to (physical row, step offset);
//      the group runs a.giters[g] steps from its rows' chunk state and saves it at the end; P1
//      and the noise are read at the row's own step, labels / logits written there.
template <int NR, int MODE, bool ROT, bool DBG>
__device__ __forceinline__ void gen_body(const PersistGenArgs& a, float* lds, const int g, const int w) {
    static_assert(!(ROT && MODE == 2), "rotated geneing launches are BITS or MOL");
    const int tid = threadIdx.x;
    const int g0 = a.rb + g;
    const int t1g = ROT ? __builtin_amdgcn_readfirstlane(a.giters[g]) : a.t1;
    auto vmap_g = [&](int r) -> int2 { return ROT ? a.vmap[g0 + kPG * r] : make_int2(g0 + kPG * r, 0); };
    const int q = tid >> 7;
    const int og = (tid >> 4) & 7, kc = tid & 15;
    const int u = GU * w + og;                  // GRU unit of quad 0's weight rows
    const int o = GO * w + og;                  // fc1 output of quad 1 (og < GO)
    const int cl = 8 * q + og;                  // fc3 class within the slot
    const int cls = a.cpw * w + cl;
    const bool has_cls = cl < a.cpw && cls < a.n_classes;
    const int j = tid & (GH - 1), hs = tid >> 8;  // GRU1: unit j of rows r = 2 i + hs
    constexpr int NRH = (NR + 1) / 2;
    const rsrc_t xr = mk_rsrc(a.xbuf + (size_t)g * QX_GROUP);

    float4 wr[kGNW];
    {
        const float4* src = a.wreg + ((size_t)w * kPT + tid) * kGNW;
#pragma unroll
        for (int i = 0; i < kGNW; ++i) wr[i] = src[i];
    }
    const size_t SW = 2 * GH;
    float h1[NRH];
#pragma unroll
    for (int i = 0; i < NRH; ++i) {
        const int r = 2 * i + hs;
        h1[i] = 0.f;
        if (r < NR) {
            const float* st = a.st + (size_t)vmap_g(r).x * SW;
            h1[i] = st[GH + j];
            lds[L_XA + r * GH + j] = st[j];
            lds[L_H1 + r * GH + j] = h1[i];
        }
    }
    if (tid < 24) lds[L_CB + tid] = a.b_hh1[(tid >> 3) * GH + GU * w + (tid & 7)];
    if (tid < NR) {
        reinterpret_cast<RowInfo*>(lds + L_RI)[tid] = a.rows[g0 + kPG * tid];
        reinterpret_cast<int2*>(lds + L_VM)[tid] = vmap_g(tid);
    }
    if (tid == 0) lds[L_FAIL] = 0.f;
    const bool own = kc < NR;
    const int lr = own ? kc : 0;
    const int2 lvm = vmap_g(lr);  // (physical row, step offset) of this lane's epilogue row
    const int lrow = lvm.x;
    const float vj0 = a.v[j], vj1 = a.v[GH + j], vj2 = a.v[2 * GH + j], w0j = a.w0[j];
    const float bcls = has_cls ? a.b_f3[cls] : 0.f;
    const rsrc_t fcr = mk_rsrc(a.fcond);
    const unsigned o_tid = (unsigned)j * 4u;
    __syncthreads();

    const float4* XA = reinterpret_cast<const float4*>(lds + L_XA);
    const float4* H1 = reinterpret_cast<const float4*>(lds + L_H1);
    const float4* Y = reinterpret_cast<const float4*>(lds + L_Y);
    float* sink = lds + L_DUMMY;
    const int wave = tid >> 6;

    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[0] = p_now();
    for (int t = a.t0; t < t1g; ++t) {
        const unsigned seq = (unsigned)t + 1u;
        const bool nxt = t + 1 < a.S;
        // ---- per-step loads: fc1 conditioning, noise, P1 / cI of step t+1 -------------------
        // (rotated: the RowInfo table by virtual row carries the row's offset in rel0)
        float pc = 0.f, pgum = 0.f;
        if (own) {
            const RowInfo& lri = reinterpret_cast<const RowInfo*>(lds + L_RI)[kc];
            if (q == 1 && og < GO)
                pc = bld(fcr, (unsigned)(p_frame(lri, t, a.hop) * a.cond_width + a.oF1 + o) * 4u, 0);
            if (has_cls && MODE == 0) {
                if constexpr (ROT)  // (the row's own step; the stream < 4 GiB, runtime-checked)
                    pgum = bld(mk_rsrc(a.gumbel),
                               (unsigned)((((unsigned)(t + lvm.y) * (unsigned)a.B + (unsigned)lrow) * (unsigned)a.n_classes +
                                           (unsigned)cls) * 4u), 0);
                else
                    pgum = bld(mk_rsrc(a.gumbel + (size_t)t * a.B * a.n_classes),
                               (unsigned)(lrow * a.n_classes + cls) * 4u, 0);
            }
        }
        // MOL: sampling lane (row tid / 32, k = tid % 32 < 11) holds draw k of its row
        if (MODE == 1 && tid < 32 * NR && (tid & 31) < 11) {
            size_t ro = (size_t)t * a.B + g0 + kPG * (tid >> 5);
            if constexpr (ROT) {  // (the row's own step)
                const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[tid >> 5];
                ro = (size_t)(t + vm.y) * a.B + vm.x;
            }
            pgum = bld(mk_rsrc(a.gumbel + ro * kMolNoise), (unsigned)(tid & 31) * 4u, 0);
        }
        float pP[NRH][3], pC[NRH];
        {  // (unconditional, step clamped: every path to the back edge consumes these loads)
            const int tn = nxt ? t + 1 : t;
            // P1 is [step][row][unit][r, z, n, cI]: one 16-byte load per row
            const rsrc_t pr = mk_rsrc(a.P1 + ((size_t)tn * a.B + g0) * 4 * GH);
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
                            mk_rsrc(a.P1 + ((size_t)ts * a.B + px) * 4 * GH), o_tid * 4u, 0, 0);
                    } else {
                        v = __builtin_amdgcn_raw_buffer_load_b128(pr, o_tid * 4u, (unsigned)(r * kPG * 4 * GH) * 4u, 0);
                    }
                    pP[i][0] = __uint_as_float(v.x);
                    pP[i][1] = __uint_as_float(v.y);
                    pP[i][2] = __uint_as_float(v.z);
                    pC[i] = __uint_as_float(v.w);
                }
            }
        }
        // ================= stage 1: q1 fc1 (critical) | q0 gh1 = W_hh1 h1 + b ===============
        if (q == 1) {
            __builtin_amdgcn_s_setprio(2);
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                v2f acc = {0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 4; ++i) dot4(acc, wr[i], XA[r * GK4 + 16 * i + kc]);
                const float tt = row16_sum(hsum(acc));
                if (kc == r) s = tt;
            }
            if (own && og < GO) {
                const float y = p_add(s, pc);
                bst_tag(y > 0.f ? y : 0.f, seq, xr, (unsigned)(lr * GF + o) * 8u, QX_Y * 4);
            }
            __builtin_amdgcn_s_setprio(0);
        } else if (q == 0) {
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                v2f acc[3] = {(v2f){0.f, 0.f}, (v2f){0.f, 0.f}, (v2f){0.f, 0.f}};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const float4 x4 = H1[r * GK4 + 16 * i + kc];
#pragma unroll
                    for (int jg = 0; jg < 3; ++jg) dot4(acc[jg], wr[4 * jg + i], x4);
                }
                const float t0 = row16_sum(hsum(acc[0]));
                const float t1 = row16_sum(hsum(acc[1]));
                const float t2 = row16_sum(hsum(acc[2]));
                if (kc == r) {
                    s0 = t0;
                    s1 = t1;
                    s2 = t2;
                }
            }
            if (own) {
                const float* cb = lds + L_CB;
                const unsigned ob = (unsigned)(lr * 3 * GH + u) * 8u;
                bst_tag(p_add(s0, cb[og]), seq, xr, ob, QX_GH * 4);
                bst_tag(p_add(s1, cb[8 + og]), seq, xr, ob + GH * 8, QX_GH * 4);
                bst_tag(p_add(s2, cb[16 + og]), seq, xr, ob + 2 * GH * 8, QX_GH * 4);
            }
        }
        if (!poll_rows<NR, GF>(xr, QX_Y * 4, seq, lds + L_Y, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
        __syncthreads();
        // ================= stage 2: fc3 -> candidates; gh1 of this step into LDS ===========
        {
            float s0 = 0.f;
            if (8 * q < a.cpw) {  // wave-uniform skip of quads without classes
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    v2f acc = {0.f, 0.f};
#pragma unroll
                    for (int i = 0; i < 2; ++i) dot4(acc, wr[12 + i], Y[r * GFK4 + 16 * i + kc]);
                    const float tt = row16_sum(hsum(acc));
                    if (kc == r) s0 = tt;
                }
            }
            // [cl][r] (logit, noise word): wave 0 forms the candidate keys (cand_key) as it
            // reduces them; MOL / BETA: the logit, published after the gh1 poll below
            float* red = lds + L_RED;
            if (own) {
                float l = -INFINITY;
                if (has_cls) {
                    l = p_add(s0, bcls);
                    p_dbg_logit<DBG>(a.dbg, t + lvm.y, lrow, cls, a.B, a.n_classes, l);
                }
                *reinterpret_cast<float2*>(red + (cl * GNR + kc) * 2) = make_float2(l, pgum);
            }
            // this step's gh1 pairs, read before this workgroup's candidate can be seen (a
            // producer overwrites them only after every candidate of this step is out)
            if (!poll_rows<NR, 3 * GH>(xr, QX_GH * 4, seq, lds + L_GH, sink, a.ctl, tid)) lds[L_FAIL] = 1.f;
            __syncthreads();
            if (wave == 0) {
                if (MODE == 0) {
                    // slot candidate per row: the max key, tagged with the step
                    const unsigned tag = key_tag(seq);
                    if (a.cpw <= 16) {
                        const int r = tid >> 4, oo = tid & 15;
                        uint32_t bh = 0, bl = 0;
                        if (r < NR && oo < a.cpw && a.cpw * w + oo < a.n_classes) {
                            const float2 lg = *reinterpret_cast<const float2*>(red + (oo * GNR + r) * 2);
                            const CandKey k = cand_key(lg.x, __float_as_uint(lg.y), a.cpw * w + oo);
                            bh = k.hi;
                            bl = k.lo;
                        }
                        row16_kmax(bh, bl);
                        if (r < NR && oo == 0)
                            __builtin_amdgcn_raw_buffer_store_b64((u2v){bh, bl | tag}, xr,
                                                                  (unsigned)((w * GNR + r) * 2) * 4u, QX_D * 4, 0);
                    } else {
#pragma unroll
                        for (int rb = 0; rb < NR; rb += 2) {
                            const int r = rb + (tid >> 5), oo = tid & 31;
                            uint32_t bh = 0, bl = 0;
                            if (r < NR && oo < a.cpw && a.cpw * w + oo < a.n_classes) {
                                const float2 lg = *reinterpret_cast<const float2*>(red + (oo * GNR + r) * 2);
                                const CandKey k = cand_key(lg.x, __float_as_uint(lg.y), a.cpw * w + oo);
                                bh = k.hi;
                                bl = k.lo;
                            }
                            half_kmax(bh, bl);
                            if (r < NR && oo == 31)
                                __builtin_amdgcn_raw_buffer_store_b64((u2v){bh, bl | tag}, xr,
                                                                      (unsigned)((w * GNR + r) * 2) * 4u, QX_D * 4, 0);
                        }
                    }
                } else {
                    // MOL / BETA: the slot's logits (row r, class c) as tagged pairs, polled
                    // directly by every workgroup's sampling lanes (after this workgroup's gh1
                    // poll, like the RAW candidates: the gh1 area is single-buffered)
                    const int r = tid >> 4, c = tid & 15;
                    if (r < NR && c < a.cpw && a.cpw * w + c < a.n_classes)
                        bst_tag(red[(c * GNR + r) * 2], seq, xr, (unsigned)(r * 32 + a.cpw * w + c) * 8u,
                                (QX_D + QX_D_LOG) * 4);
                }
            }
        }
        // ================= sample of step t (redundant in every workgroup) ==================
        if (MODE == 0) {
            if (tid < 32 * NR) {
                const int r = tid >> 5, oo = tid & 31;
                const unsigned off = (unsigned)((oo * GNR + r) * 2) * 4u;
                const unsigned want = key_tag(seq);
                u2v c;
                const unsigned ts = p_now();
                unsigned n = 0;
                while (true) {
                    c = __builtin_amdgcn_raw_buffer_load_b64(xr, off, QX_D * 4, kCpNT);
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
                if (oo == 31) {
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
            // MOL / BETA: half-wave r, lane k polls logit k of row r (tagged pair)
            const int r = tid >> 5, k = tid & 31, row = g0 + kPG * r;
            const unsigned so = (QX_D + QX_D_LOG) * 4;
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
            float xv = 0.f;
            if (MODE == 2) {
                // BETA (geneing 'RAW'): vocoder/distribution.py:7-20, Beta(exp l0, exp l1) on
                // [-1, 1] with the Philox gamma draws (philox.h beta_sample)
                // [-1, 1] with the Philox gamma draws: lane 0 draws X ~ Gamma(exp l0), lane 1
                // Y ~ Gamma(exp l1) concurrently (philox.h gamma_mt, g = lane); lane 0 forms
                // 2 X / (X + Y) - 1 exactly as beta_sample does
                double gv = 0.0;
                if (k < 2) {
                    const RowInfo& lri = reinterpret_cast<const RowInfo*>(lds + L_RI)[r];
                    gv = gamma_mt((double)expf(lk), (uint32_t)k, (uint32_t)t, (uint32_t)lri.fold,
                                  lri.stream, a.k0, a.k1);
                }
                const double gy = __shfl(gv, base + 1);
                if (k == 0) {
#pragma clang fp contract(off)
                    const float sb = (float)(gv / (gv + gy));
                    xv = 2.0f * sb - 1.0f;
                }
            } else {
                // MOL: vocoder/distribution.py:104-140; lane k holds draw k of k_mol_noise
                // (gm_k = log(-log(u1_k)), k < 10; gm_10 = log(u2) - log(1 - u2))
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
                {
#pragma clang fp contract(off)
                    const float lsmin = -32.23619130191664f;  // float(np.log(1e-14))
                    ls = ls < lsmin ? lsmin : ls;
                    xv = mean + expf(ls) * lu;
                    xv = xv < -1.f ? -1.f : xv;
                    xv = xv > 1.f ? 1.f : xv;
                }
            }
            if (k == 0) {
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
                const float* gh = lds + L_GH + r * 3 * GH + j;
                const float hn = p_gru(fmaf(vj0, x, pP[i][0]), fmaf(vj1, x, pP[i][1]),
                                       fmaf(vj2, x, pP[i][2]), gh[0], gh[GH], gh[2 * GH], h1[i]);
                h1[i] = hn;
                lds[L_XA + r * GH + j] = p_add(fmaf(w0j, x, pC[i]), hn);
                lds[L_H1 + r * GH + j] = hn;
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
    if ((ROT || a.t1 < a.S) && w == 0) {
#pragma unroll
        for (int i = 0; i < NRH; ++i) {
            const int r = 2 * i + hs;
            if (r < NR) {
                float* st = a.st + (size_t)vmap_g(r).x * SW;
                st[j] = lds[L_XA + r * GH + j];
                st[GH + j] = lds[L_H1 + r * GH + j];
            }
        }
    }
}

template <int NR, int MODE, bool ROT, bool DBG>
__global__ __launch_bounds__(kPT, 1) void k_persist_gen(PersistGenArgs a) {
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
            gen_body<NR, MODE, true, DBG>(a, lds, g, w);
        else
            gen_body<NR - 1, MODE, true, DBG>(a, lds, g, w);
    } else {
        gen_body<NR, MODE, false, DBG>(a, lds, g, w);
    }
}

// Step-0 state: GRU1 with x = 0, h = 0 (gh = b_hh1) -> x1(0), h1(0).
__global__ __launch_bounds__(kRH) void k_persist_gen_init(PersistGenArgs a) {
    const int row = blockIdx.x, j = threadIdx.x, H = GH;
    const float* P1 = a.P1 + ((size_t)row * H + j) * 4;  // step 0: (r, z, n, cI) of unit j
    const float hn = p_gru(P1[0], P1[1], P1[2], a.b_hh1[j], a.b_hh1[H + j], a.b_hh1[2 * H + j], 0.f);
    float* st = a.st + (size_t)row * 2 * H;
    st[j] = p_add(P1[3], hn);
    st[H + j] = hn;
}

hipError_t launch_persist_gen_init(const PersistGenArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_persist_gen_init, dim3(a.B), dim3(GH), 0, s, a);
    return hipGetLastError();
}

// at least 96 KB so that no CU can take two workgroups of this (register-light) kernel:
// every group must span 32 CUs
size_t persist_gen_lds_bytes() {
    const size_t need = (size_t)L_TOTAL * sizeof(float);
    return need > 96 * 1024 ? need : 96 * 1024;
}
size_t persist_gen_xbuf_floats() { return (size_t)kPG * QX_GROUP; }

// Each sampling mode is its own instantiation: the BETA float64 gamma sampler would otherwise
// raise the register allocation of the RAW / MOL variants
template <int NR, int MODE>
hipError_t launch_persist_gen_t(const PersistGenArgs& a, hipStream_t s) {
    if constexpr (MODE != 2 && NR >= 2) {
        if (a.vmap) {  // rotated (BITS / MOL, 2-4 rows per group)
            if (a.dbg.out) return persist_launch<k_persist_gen<NR, MODE, true, true>>(persist_gen_lds_bytes(), a, s);
            return persist_launch<k_persist_gen<NR, MODE, true, false>>(persist_gen_lds_bytes(), a, s);
        }
    }
    if (a.vmap) return hipErrorInvalidValue;
    if (a.dbg.out) return persist_launch<k_persist_gen<NR, MODE, false, true>>(persist_gen_lds_bytes(), a, s);
    return persist_launch<k_persist_gen<NR, MODE, false, false>>(persist_gen_lds_bytes(), a, s);
}

template <int NR, int MODE>
int persist_gen_spill_t() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_persist_gen<NR, MODE, false, false>) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}

// scratch bytes of the rotated BITS (mode 0) / MOL (1) instance of nr (2-4) rows per group; -1 if none
int persist_gen_rot_scratch(int nr, int mode) {
    hipFuncAttributes fa;
    const void* f = nullptr;
    if (mode == 0)
        f = nr == 2 ? (const void*)k_persist_gen<2, 0, true, false>
          : nr == 3 ? (const void*)k_persist_gen<3, 0, true, false>
          : nr == 4 ? (const void*)k_persist_gen<4, 0, true, false> : nullptr;
    else if (mode == 1)
        f = nr == 2 ? (const void*)k_persist_gen<2, 1, true, false>
          : nr == 3 ? (const void*)k_persist_gen<3, 1, true, false>
          : nr == 4 ? (const void*)k_persist_gen<4, 1, true, false> : nullptr;
    if (!f || hipFuncGetAttributes(&fa, f) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}

template <int MODE>
int persist_gen_spill_nr(int nr) {
    switch (nr) {
        case 1: return persist_gen_spill_t<1, MODE>();
        case 2: return persist_gen_spill_t<2, MODE>();
        case 3: return persist_gen_spill_t<3, MODE>();
        case 4: return persist_gen_spill_t<4, MODE>();
        default: return -1;
    }
}

int persist_gen_variant_ok(int nr, int cpw, int mode) {
    if (cpw < 1 || cpw > 32 || (mode != 0 && cpw > 16)) return 0;
    // (the BETA variants keep a small stack frame for the float64 trig range reduction)
    const int sp = mode == 2 ? persist_gen_spill_nr<2>(nr)
                 : mode == 1 ? persist_gen_spill_nr<1>(nr) : persist_gen_spill_nr<0>(nr);
    return sp >= 0 && sp <= (mode == 2 ? 16 : 0) ? 1 : 0;
}

template <int MODE>
hipError_t launch_persist_gen_m(const PersistGenArgs& a, hipStream_t s) {
    switch (a.nr) {
        case 1: return launch_persist_gen_t<1, MODE>(a, s);
        case 2: return launch_persist_gen_t<2, MODE>(a, s);
        case 3: return launch_persist_gen_t<3, MODE>(a, s);
        case 4: return launch_persist_gen_t<4, MODE>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_persist_gen(const PersistGenArgs& a, hipStream_t s) {
    if (a.rb < 0 || a.nr < 1 || a.rb + kPG * a.nr > a.B || a.cpw < 1 || a.cpw > 32 ||
        a.cpw * kPM < a.n_classes || (a.mode != 0 && (a.n_classes > 32 || a.cpw > 16)))
        return hipErrorInvalidValue;
    return a.mode == 2 ? launch_persist_gen_m<2>(a, s)
         : a.mode == 1 ? launch_persist_gen_m<1>(a, s) : launch_persist_gen_m<0>(a, s);
}

}  // namespace wrnn
