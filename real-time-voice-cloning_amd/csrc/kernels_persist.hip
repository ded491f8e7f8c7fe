// Persistent, weight-stationary recurrence of the fatchord WaveRNN (the "persist" engine).
//
// Reference step body: vocoder/models/fatchord_version.py:192-236. One launch runs a chunk of
// steps for all fold rows. The 256 workgroups (one per CU, 512 threads) form 8 groups from the
// workgroups that report the same HW_REG_XCC_ID, so every group lives on one XCD and shares
// its L2. Group g owns fold rows rb+g, rb+g+8, ... (NR rows of one row batch; the host pads
// the row count to a multiple of 8*NR and launches once per batch)
// and holds ALL step weights, spread over its 32 workgroups (slot w owns GRU units / outputs
// [16w, 16w+16) and fc3 classes [cpw*w, cpw*(w+1))): registers hold W_ih2[:, :512] and W_hh1
// (r,z,n rows of the slot's units) and the fc1/fc2 rows; LDS holds the W_hh2 rows and the fc3
// rows (registers when a slot owns more than 16 classes, i.e. 10-bit). Nothing is re-read from
// HBM per step except the precomputed per-step inputs (P1, cI, per-frame aux terms, Gumbel
// noise), loaded a step ahead so their latency hides behind the exchanges (an explicit L2
// warm-up two steps ahead measured 5 % slower and was dropped).
//
// Per step, four in-group exchanges of tagged pairs (value, step + 1) stored to the group's
// exchange area and polled with non-temporal loads served by the XCD's shared L2:
//   A: GRU2 (W_ih2 x1 + cond, gh2 of the previous step) -> x2, h2
//   B: fc1 (relu) on x2
//   C: fc2 (relu) on y1
//   D: fc3 on y2 -> per-slot Gumbel-max candidates (RAW) or logits (MOL)
// Each of these runs alone on the CU; the off-path products run in the exchange waits that
// follow (behind a workgroup barrier): W_hh1 h1 + b -> gh1 (published) in hop A, W_hh2 h2 + b
// -> gh2 of the next step (kept local) in hops B and C. Redundantly in every workgroup: the
// sample of step t and GRU1 of step t+1 for all 512 units (so x1/h1 never need an exchange).
// Sampling: argmax_k (l_k + G_k), G_k = -log q_k with q the RNG contract's Exp(1) variate,
// G in fixed point to 2^-27 and l + G formed exactly as an fp32 pair (TwoSum, cand_key.h) --
// the reference's argmax((softmax(l)/sum)/q) without the fp32 rounding of round 4's l + g.
// Every spin is bounded; on a timeout the kernel sets an error code and every group exits.
#include "wrnn_kernels.h"
#include "persist_common.h"
#include "philox.h"

// The Makefile compiles this file twice, so that each half gets the machine-scheduler strategy
// measured fastest for it on MI355X: part 1 = the categorical (RAW) variants,
// the launch dispatch and the helper kernels, with the iterative ILP strategy; part 2 = the MOL
// variants with the default strategy (ILP spills the MOL 3-row variant). Part 0 (the default)
// is everything in one object (tools/build_variant.sh).
#ifndef WRNN_PERSIST_PART
#define WRNN_PERSIST_PART 0
#endif

namespace wrnn {

// exchange area per group (floats). A, B, C hold tagged pairs (value bits, step + 1), so a
// consumer polls the payload itself -- no flags: A double-buffered [r][x2 | h2 | gh1 r,z,n][512],
// B y1 [r][512], C y2 [r][512]; D the per-slot candidates (RAW, tagged) / MOL logits.
constexpr int XB_A = 0;
constexpr int XB_A_SZ = kPNR * 5 * kPH * 2;
constexpr int XB_B = XB_A + 2 * XB_A_SZ;
constexpr int XB_C = XB_B + kPNR * kPH * 2;
constexpr int XB_D = XB_C + kPNR * kPH * 2;
// RAW candidates [slot][r][value, tag] (the area is sized for 4 per slot and row)
constexpr int XB_D_LOG = kPM * kPNR * 4 * 2;
constexpr int XB_D_SZ = XB_D_LOG + kPNR * 64;      // MOL logits [r][64]
constexpr int XB_G = XB_D + XB_D_SZ;              // gh1 [parity][r][unit] (r, z, n, -) float4
constexpr int XB_G_SZ = 2 * kPNR * kPH * 4;
constexpr int XB_P = XB_G + XB_G_SZ;              // P1 ring [parity][r][unit] (r, z, n, cI) float4
constexpr int XB_P_SZ = 2 * kPNR * kPH * 4;
constexpr int XB_GROUP = XB_P + XB_P_SZ + 64;

// LDS carve (floats). The per-step operands come first so every ds_read offset of the inner
// loops fits the 16-bit immediate (no per-(q, row) address registers).
constexpr int L_X0 = 0;                             // [kPNR][512]
constexpr int L_X1 = L_X0 + kPNR * kPH;             // [kPNR][512] h1
constexpr int L_XH2 = L_X1 + kPNR * kPH;            // [kPNR][512] h2 (staged at hop A)
constexpr int L_RED = L_XH2 + kPNR * kPH;           // [32 og][kPNR][2]
constexpr int L_SX = L_RED + kPCls * kPNR * 2;      // sampled x per row
constexpr int L_FAIL = L_SX + 12;                   // set when a tagged poll gave up
constexpr int L_ARR = L_SX + 13;                    // stage-A arrivals of waves 0-3 (uint, monotonic)
// x2 of a launch with NR < kPNR rows per group: row r in the unused last row slot of X0 / X1 / XH2
// (row stride kPNR * kPH floats), so hop A never writes over the x1 that stage A reads
constexpr int L_X2 = L_X0 + (kPNR - 1) * kPH;
static_assert(L_X1 == L_X0 + kPNR * kPH && L_XH2 == L_X1 + kPNR * kPH &&
                  L_X2 + (kPNR - 2) * kPNR * kPH + kPH == L_XH2 + kPNR * kPH,
              "x2 rows 0 .. kPNR - 2 sit in the last row slots of X0, X1, XH2");

constexpr int L_GH2 = L_SX + 16;                    // gh2 = W_hh2 h2 + b_hh2 [16 units][3][kPNR]
constexpr int L_RI = L_GH2 + 16 * 3 * kPNR;         // RowInfo of the group's rows (6 words each)
constexpr int L_VM = L_RI + 6 * kPNR;               // (physical row, step offset) of each row slot
constexpr int L_BIAS = L_VM + 2 * kPNR;             // b_hh1, b_hh2 of the slot's units [2][3][16]
constexpr int L_W0 = L_BIAS + 96;                    // w0 = W_ih1[:, 0] [512] (GRU1 input term)
constexpr int L_BCLS = L_W0 + kPH;                  // b_fc3 of the slot's classes [32]
constexpr int L_W = (L_BCLS + kPCls + 3) & ~3;      // slot weights (kPLdsW4 float4)
constexpr int L_FC3 = L_W + 16 * 3 * kPH;           // fc3 rows inside the weight block
constexpr int L_TOTAL = L_W + 4 * kPLdsW4;
static_assert(L_W % 4 == 0, "weights must be 16-byte aligned");
static_assert(L_TOTAL * 4 + 64 <= 160 * 1024, "LDS carve exceeds the CU's 160 KiB");


// ---- sparse products (SP instances: pruned checkpoints) --------------------
// The slot's weights as its live 1 x 4 blocks (the Pruner's groups, vocoder/pruner.py:60-88) in
// LDS (runtime.hip pack_persist_sparse): per product set and 16-lane row group (one output row
// of the slot), entry e of lane kc at float4 index base + 16 e, the lane's base and masks in its
// four words of PersistArgs::wreg; mask bit 8 j + q says block q of gate j (columns
// 4 (16 q + kc) .. + 3, the dense kernel's register float4 wr[8 j + q]) is live. Each round takes
// the next live block of every gate at once; a lane with none left reads the zero row
// (kPSpZero) against block 0 of X, so its fma adds an exact zero. Every (row, gate) accumulator
// sees its live blocks in increasing q -- the dense kernel's order minus products that are exact
// zeros -- so the sums are bit-identical to the dense kernel's on the same weights.
// RM: the rows (bit r) accumulated.
template <int NR, int G, int RM = 0xF, int XSTR = kPK4>
__device__ __forceinline__ void sp_products(const float4* Wsp, const float4* Xs, unsigned (&m)[G],
                                            unsigned (&p)[G], const int kc, v2f (&acc)[NR][G]) {
    const unsigned zb = (unsigned)(kPSpZero + kc);
    while (true) {
        unsigned any = 0u;
#pragma unroll
        for (int j = 0; j < G; ++j) any |= m[j];
        if (any == 0u) break;
        unsigned q[G];
        float4 wv[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const bool v = m[j] != 0u;
            q[j] = v ? (unsigned)__builtin_ctz(m[j]) : 0u;
            m[j] &= m[j] - 1u;
            wv[j] = Wsp[v ? p[j] : zb];
            p[j] += v ? 16u : 0u;
        }
        // (fully unrolled by the compiler: constant trip counts; an explicit pragma here is
        // reported as not applied once the row mask has removed rows)
        for (int r = 0; r < NR; ++r)
            if ((RM >> r) & 1)
                for (int j = 0; j < G; ++j) dot4(acc[r][j], wv[j], Xs[r * XSTR + 16 * q[j] + kc]);
    }
}
// rows r < NR of the W_hh2 window WIN (r % 3 == WIN) as a row mask
constexpr int hh2_rowmask(int win, int nr) {
    int m = 0;
    for (int r = 0; r < nr; ++r)
        if (r % 3 == win) m |= 1 << r;
    return m;
}

// P1R: P1 from the in-launch ring (PersistArgs::p1q) instead of the [S][B][4H] stream.
// DBG: the instance that records logits for the teacher-forced gate (wrnn_set_debug_steps)
// ROT: a rotated launch (PersistArgs::vmap): row slot r of the group is the
//      virtual row v = g + 8 r, which a.vmap maps to (physical row, step offset of the launch);
//      the group runs a.giters[g] steps (its rows' steps off .. off + giters - 1). The per-launch
//      RowInfo table (a.rows, by virtual row) carries rel0 + offset, so every per-frame /
//      per-position lookup follows; noise, labels, samples, state and logits use the physical
//      row and the offset step.
// SP: the sparse instance (pruned weights, block lists in LDS; sp_products above)
template <int NR, bool FC3R, bool MOL, bool P1R, bool ROT, bool DBG, bool SP>
__device__ __forceinline__ void persist_body(const PersistArgs& a, float* lds, const int g, const int w) {
    static_assert(!ROT || P1R, "rotated launches form P1 in the ring");
    static_assert(!SP || P1R, "sparse instances form P1 in the ring");
    const int tid = threadIdx.x;
    const int g0 = a.rb + g;  // first (virtual) fold row of this group in this launch
    // the group's step range: [t0, t1) (rotated: its own step count, offsets per row)
    const int t1g = ROT ? __builtin_amdgcn_readfirstlane(a.giters[g]) : a.t1;
    // clamp of the look-ahead loads of noise / conditioning (step indices < tend; past the
    // group's last step their values go unused)
    const int tend = ROT ? t1g : a.S;
    const int og = tid >> 4, kc = tid & 15;
    constexpr int H = kPH;
    const int u = 16 * w + (og & 15);   // unit / output of this thread's weight rows
    const bool gate_a = og < 16;        // stage A: W_ih2 (og<16) | W_hh1 (og>=16)
    const int cls = a.cpw * w + og;     // fc3 class of this thread
    const bool has_cls = og < a.cpw && cls < a.n_classes;
    const rsrc_t xr = mk_rsrc(a.xbuf + (size_t)g * XB_GROUP);  // this group's exchange area
    const bool trace = a.phases != nullptr;
    uint32_t* ph = trace ? a.phases + (size_t)(g * kPM + w) * kPPhases : nullptr;
    // stamps of wave 0 at [i], of wave 4 at [12 + i]; shader-clock cycles of the traced step
    // (wave 0) at [24] / [25] give the core clock against the 100 MHz stamps
#define XSTAMP(i)                                                        \
    if (trace && t == a.phase_t && tid == 0) ph[(i)] = p_now();
    // float4 per row per LDS batch of the 3-gate / 1-gate products (2 / 2 fastest)
    constexpr int kPQB3 = 2, kPQB1 = 2;
#define PSTAMP(i)                                                        \
    if (trace && t == a.phase_t && (tid & 255) == 0) {                   \
        ph[(tid >> 8) * 12 + (i)] = p_now();                             \
        if (tid == 0 && ((i) == 0 || (i) == 10))                         \
            ph[24 + ((i) == 10)] = (uint32_t)__builtin_amdgcn_s_memtime(); \
    }

    // ---- weights: registers and LDS -----------------------------------------------------
    constexpr int NW = SP ? 1 : FC3R ? 40 : 32;
    float4 wr[NW];
    // SP: the lane's masks and list bases (x: set A | fc << 24, y: W_hh2 | fc3 << 24,
    // z / w: their bases, 16 bits each) -- the whole slot image goes to LDS
    uint4 si = make_uint4(0u, 0u, 0u, 0u);
    {
        if constexpr (SP) {
            si = reinterpret_cast<const uint4*>(a.wreg)[(size_t)w * kPT + tid];
        } else {
            const float4* src = a.wreg + ((size_t)w * kPT + tid) * NW;
#pragma unroll
            for (int i = 0; i < NW; ++i) wr[i] = src[i];
        }
        const float4* hs = a.wlds + (size_t)w * kPLdsW4;
        float4* hd = reinterpret_cast<float4*>(lds + L_W);
        const int n4 = FC3R && !SP ? 16 * 3 * kPK4 : kPLdsW4;
        for (int i = tid; i < n4; i += kPT) hd[i] = hs[i];
    }
    const float4* Wsp = reinterpret_cast<const float4*>(lds + L_W);
    // ---- chunk state -----------------------------------------------------------------------
    // thread tid = unit j of the redundant GRU1; lanes kc < NR of og < 16 own (u, row kc) of GRU2
    float h1[NR], h2r = 0.f;
    const bool own = gate_a && kc < NR;
    const int lr = kc < NR ? kc : 0;
    // physical row / step offset of row slot r (identity / 0 unless rotated)
    auto vmap_g = [&](int r) -> int2 { return ROT ? a.vmap[g0 + kPG * r] : make_int2(g0 + kPG * r, 0); };
    const int2 lvm = vmap_g(lr);
    const int lrow = lvm.x;  // (physical) row of this lane's epilogue
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const int row = vmap_g(r).x;
        h1[r] = a.st_h1[(size_t)row * H + tid];
        lds[L_X0 + r * kPH + tid] = a.st_x1[(size_t)row * H + tid];
        lds[L_X1 + r * kPH + tid] = h1[r];
    }
    if (own) {
        h2r = a.st_h2[(size_t)lrow * H + u];
#pragma unroll
        for (int j = 0; j < 3; ++j)
            lds[L_GH2 + (og * 3 + j) * kPNR + kc] = a.st_gh2[(size_t)lrow * 3 * H + j * H + u];
    }
    // per-thread constants
    // (w0 and b_fc3 wait in LDS: read once per step each, they need no register)
    const float vj0 = a.v[tid], vj1 = a.v[H + tid], vj2 = a.v[2 * H + tid];
    lds[L_W0 + tid] = a.w0[tid];
    if (tid < 96) lds[L_BIAS + tid] = (tid < 48 ? a.b_hh1 : a.b_hh2)[(tid % 48 / 16) * H + 16 * w + (tid & 15)];
    if ((tid & 15) == 0) lds[L_BCLS + og] = has_cls ? a.b_fc3[cls] : 0.f;
    if (tid < NR) {
        reinterpret_cast<RowInfo*>(lds + L_RI)[tid] = a.rows[g0 + kPG * tid];
        reinterpret_cast<int2*>(lds + L_VM)[tid] = vmap_g(tid);
    }
    // per-lane byte offsets (32-bit)
    const unsigned o_tid = (unsigned)tid * 4u;                          // unit tid of a row
    const unsigned o_u = (unsigned)(lr * 5 * kPH + u) * 8u;             // bufA pair (row lr, unit u)
    const unsigned o_y = (unsigned)(lr * kPH + u) * 8u;                 // bufB/C pair (row lr, unit u)
    // gumbel row lrow (a padding row reads row rb's: no HBM traffic for padding); a rotated
    // launch reads its rows' steps off + t: the offset folded into the lane's base
    const unsigned o_gum = ROT ? (unsigned)(((lvm.y * a.B) + lrow) * a.n_classes + cls) * 4u
                               : (unsigned)((lrow < a.nreal ? lrow : a.rb) * a.n_classes + cls) * 4u;
    const rsrc_t fcr = mk_rsrc(a.fcond);
    __syncthreads();

    const float4* X0 = reinterpret_cast<const float4*>(lds + L_X0);
    const float4* X1 = reinterpret_cast<const float4*>(lds + L_X1);
    const float4* XH2 = reinterpret_cast<const float4*>(lds + L_XH2);
    // x2 (fc1's input): its own rows below kPNR rows per group (L_X2); at kPNR rows formed in
    // place over x1 in X0, after the hop-A arrival guard
    constexpr bool X2B = NR < kPNR;
    const float4* X2 = reinterpret_cast<const float4*>(lds + (X2B ? L_X2 : L_X0));
    constexpr int X2S = X2B ? kPNR * kPK4 : kPK4;  // its row stride (float4)
    const int wave = tid >> 6;
    const bool wv_lo = wave < 4;  // waves 0-3: og < 16 (GRU2, hh2, fc2, fc3 <= 16 classes)
    // Per-step operands, issued right after the wave's last publish of the previous step
    // (waves 0-3: hop C, waves 4-7: hop B) so the publish never waits on them:
    //   pP/pC  P1(tg+1), cI(tg+1) of this thread's GRU1 unit   (end of step tg)
    //   pc*    per-frame conditioning of step te's epilogues  (stages A-C of step te)
    //   pgn    noise of step te, class cls (copied to pgum at the end of step te-1)
    float pP[NR][3], pC[NR];
    float pc0 = 0.f, pc1 = 0.f, pc2 = 0.f, pf2 = 0.f;
    // pgn / pgum: RAW -- the lane's Gumbel noise in the contract's fixed-point form (k_gumbel,
    // philox.h gumbel_q_of: G = -log q to 2^-27, as a 32-bit word in a float register);
    // MOL -- the lane's draw of k_mol_noise
    float pgum = 0.f, pgn = 0.f;    // At <= 16 classes per slot waves 4-7 hold no fc3 class: they issue their GRU1 loads
    // while waves 0-3 compute fc3 (LDS only) and later poll the candidates; waves 0-3
    // issue theirs after the candidate publish, off the critical path (a wave polls only
    // with no bulk loads in flight: its first poll would wait for all of them).
    constexpr bool EARLY = !FC3R;  // sampling lanes: st = EARLY ? tid - 256 : tid in [0, 32 NR)
    // local x2 (RAW): hop A carries h2 only and every slot forms x2 = x1 + h2 itself (see hop
    // A); MOL publishes x2 (measured 6.28 vs 6.24 us per step with the local form)
    constexpr bool X2L = !MOL;
    // Loads are unconditional (step indices clamped; past the last step the values go
    // unused): every path to the loop's back edge then consumes them, so the compiler's
    // wait insertion sees no load pending at the top of the step.
    // P1R producer lanes: waves 4-7 (og >= 16), lane kc < 4 NR forms component kc % 4 of P1
    // (row kc / 4, unit u) of step t + 2 from the per-frame projections: the taps of its phase
    // and the five frame rows around its frame, loaded with the step's GRU1 operands
    const bool p1own = P1R && !gate_a && kc < 4 * NR;
    float pk = 0.f, pq[4], pa = 0.f;  // pk: tap (kc % 4) of the phase, quad-broadcast at use
    auto p1_loads = [&](int tau) {  // operands of P1(tau) for this producer lane
        if (!p1own) return;
        int tx = tid;  // (lane offsets recomputed per step: hoisted ones cost registers)
        asm volatile("" : "+v"(tx));
        const int kx = tx & 15, ux = 16 * w + ((tx >> 4) & 15);
        const RowInfo& ri = reinterpret_cast<const RowInfo*>(lds + L_RI)[kx >> 2];
        // (a row's own steps end at S: a rotated row at offset off reads P1 up to S - 1 - off;
        // the P1 of the step after the launch's last one feeds the GRU1 whose state is saved)
        const int lim = ROT ? a.S - reinterpret_cast<const int2*>(lds + L_VM)[kx >> 2].y : a.S;
        tau = tau < lim ? tau : lim - 1;
        const unsigned p = (unsigned)(ri.rel0 + tau);
        const bool in = p < (unsigned)ri.L;  // else the zero tail pad: bias only (zero frame)
        const unsigned f = p / (unsigned)a.hop, sph = in ? p - f * (unsigned)a.hop : 0u;
        // frame slots (runtime.hip): zero frame at fbase, frame j at fbase + 1 + j, zero guard
        // slots at fbase - 1 and fbase + T + 1, + 2: the phase's 4 frames need no bounds check
        const unsigned s0 = in ? (unsigned)ri.fbase - 1u + f + (sph >= (unsigned)a.p1split ? 1u : 0u)
                               : (unsigned)ri.fbase;
        const unsigned col = (unsigned)(4 * ux + (kx & 3)) * 4u;
        // the 4 lanes of a row (one DPP quad) load its 4 taps, one each
        pk = bld(mk_rsrc(a.p1taps), (sph * 4u + (unsigned)(kx & 3)) * 4u, 0);
        const rsrc_t qr = mk_rsrc(a.p1q);
        constexpr unsigned kRow = 4u * kPH * 4u;  // bytes per frame slot
#pragma unroll
        for (int k = 0; k < 4; ++k) pq[k] = bld(qr, (in ? s0 + (unsigned)k : s0) * kRow + col, 0);
        pa = bld(mk_rsrc(a.p1a), (in ? (unsigned)ri.fbase + 1u + f : s0) * kRow + col, 0);
    };
    // P1(tau) into ring slot tau & 1: k_p1_expand's fma chain without its zero taps, so the
    // same values as the stream
    auto p1_store = [&](int tau) {
        if (!p1own) return;
        float m = 0.f;  // tap k from quad lane k (quad_perm(k, k, k, k))
        m = fmaf(pdpp<0x00>(pk), pq[0], m);
        m = fmaf(pdpp<0x55>(pk), pq[1], m);
        m = fmaf(pdpp<0xAA>(pk), pq[2], m);
        m = fmaf(pdpp<0xFF>(pk), pq[3], m);
        int tx = tid;
        asm volatile("" : "+v"(tx));
        const int kx = tx & 15, ux = 16 * w + ((tx >> 4) & 15);
        const unsigned o = (unsigned)((((tau & 1) * kPNR + (kx >> 2)) * kPH + ux) * 4 + (kx & 3)) * 4u;
        bst(p_add(m, pa), xr, o, XB_P * 4);
    };
    auto prefetch = [&](int tg, int te) {
        if constexpr (!P1R) {  // P1 is [step][row][unit][r, z, n, cI]: one 16-byte load per row
            const int tn = tg + 1 < a.S ? tg + 1 : a.S - 1;
            const rsrc_t pr = mk_rsrc(a.P1 + ((size_t)tn * a.B + a.rb) * 4 * H);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                // (a padding row reads row rb's P1: same lines as a real row, no HBM traffic)
                const int rw = g0 + kPG * r < a.nreal ? g0 - a.rb + kPG * r : 0;
                const u4v v = __builtin_amdgcn_raw_buffer_load_b128(pr, o_tid * 4u,
                                                                     (unsigned)(rw * 4 * H) * 4u, 0);
                pP[r][0] = __uint_as_float(v.x);
                pP[r][1] = __uint_as_float(v.y);
                pP[r][2] = __uint_as_float(v.z);
                pC[r] = __uint_as_float(v.w);
            }
        }
        te = te < tend ? te : tend - 1;
        if (kc < NR) {
            int uu = u;  // (offsets recomputed per step: hoisted ones cost registers)
            asm volatile("" : "+v"(uu));
            const unsigned o_fc = (unsigned)((gate_a ? a.oG2 : a.oF1) + uu) * 4u;
            const unsigned o_f2 = (unsigned)(a.oF2 + uu) * 4u;
            const RowInfo& lri = reinterpret_cast<const RowInfo*>(lds + L_RI)[kc];
            const unsigned fo = (unsigned)(p_frame(lri, te, a.hop) * a.cond_width) * 4u;
            pc0 = bld(fcr, o_fc + fo, 0);
            if (gate_a) {
                pc1 = bld(fcr, o_fc + fo, H * 4);
                pc2 = bld(fcr, o_fc + fo, 2 * H * 4);
                pf2 = bld(fcr, o_f2 + fo, 0);
            }
            if (has_cls && !MOL)
                pgn = bld(mk_rsrc(a.gumbel + (size_t)te * a.B * a.n_classes), o_gum, 0);
        }
        // MOL: sampling lane (row r, k < 11) holds draw k of its row (k_mol_noise)
        if (MOL) {
            const int sl = EARLY ? tid - 256 : tid;
            if (sl >= 0 && sl < 32 * NR && (sl & 31) < 11) {
                const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[sl >> 5];
                const int mrow = ROT ? vm.x : (vm.x < a.nreal ? vm.x : a.rb);
                pgn = bld(mk_rsrc(a.gumbel + ((size_t)(te + vm.y) * a.B + mrow) * kMolNoise),
                          (unsigned)(sl & 31) * 4u, 0);
            }
        }
    };
    if (tid == 0) {
        lds[L_FAIL] = 0.f;
        reinterpret_cast<unsigned*>(lds)[L_ARR] = 0u;
    }
    if constexpr (P1R) {  // ring prologue: P1(t0 + 1), read by GRU1 of step t0
        __syncthreads();  // RowInfo in LDS
        p1_loads(a.t0 + 1);
        p1_store(a.t0 + 1);
    }
    prefetch(a.t0, a.t0);
    pgum = pgn;
    __syncthreads();
    const int tl = tid & 255;  // index inside the half that stages
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[0] = p_now();
    for (int t = a.t0; t < t1g; ++t) {
        const unsigned seq = (unsigned)t + 1u;
        const unsigned sA = (unsigned)(XB_A + (t & 1) * XB_A_SZ) * 4u;  // bufA of this step
        PSTAMP(0);
        // Each matrix-vector product on the critical path runs alone on the CU: the off-path
        // ones (W_hh1 h1, W_hh2 h2) are placed behind a workgroup barrier into the exchange
        // waits that follow it, so they never compete for VALU issue or LDS bandwidth.
        // 3-gate product of this thread's register rows (wr[0..23]) with the rows of Xs
        // Matrix-vector products: k-outer in batches of QB float4 per row with every row's
        // loads of a batch in flight together (one LDS round trip per batch, not per row);
        // each row still accumulates in k order, as a row-outer loop would.
        auto mv3 = [&](const float4* Xs, float& s0, float& s1, float& s2) {
            constexpr int QB = NR >= 4 ? 1 : kPQB3;
            v2f acc[NR][3];
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[r][j] = (v2f){0.f, 0.f};
            if constexpr (SP) {
                const unsigned mx = si.x, pb = si.z & 0xffffu;
                unsigned m[3] = {mx & 0xffu, (mx >> 8) & 0xffu, (mx >> 16) & 0xffu};
                const unsigned c0 = (unsigned)__builtin_popcount(m[0]), c1 = (unsigned)__builtin_popcount(m[1]);
                unsigned p[3] = {pb, pb + 16u * c0, pb + 16u * (c0 + c1)};
                sp_products<NR, 3>(Wsp, Xs, m, p, kc, acc);
            } else
#pragma unroll
            for (int qb = 0; qb < 8; qb += QB) {
                __builtin_amdgcn_sched_barrier(0);
                float4 xq[NR][QB];
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int q = 0; q < QB; ++q) xq[r][q] = Xs[r * kPK4 + 16 * (qb + q) + kc];
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int q = 0; q < QB; ++q)
#pragma unroll
                        for (int j = 0; j < 3; ++j) dot4(acc[r][j], wr[j * 8 + qb + q], xq[r][q]);
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float t0 = row16_sum(hsum(acc[r][0]));
                const float t1 = row16_sum(hsum(acc[r][1]));
                const float t2 = row16_sum(hsum(acc[r][2]));
                if (kc == r) {
                    s0 = t0;
                    s1 = t1;
                    s2 = t2;
                }
            }
        };
        // ================= stage A: GRU2 (waves 0-3, critical) | W_hh1 h1 + b -> gh1 (4-7) ====
        {
            // GRU2 waves first on each SIMD (a W_hh1 wave shares it; gh1 is needed only at GRU1)
            if (gate_a) __builtin_amdgcn_s_setprio(2);
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            mv3(gate_a ? X0 : X1, s0, s1, s2);
            XSTAMP(29);
            if (kc < NR) {
                if (gate_a) {
                    const float* gh2 = lds + L_GH2 + og * 3 * kPNR + kc;
                    const float hn = p_gru(p_add(s0, pc0), p_add(s1, pc1), p_add(s2, pc2),
                                           gh2[0], gh2[kPNR], gh2[2 * kPNR], h2r);
                    h2r = hn;
                    if (!X2L)  // (X2_LOCAL: every slot forms x2 = x1 + h2 itself)
                        bst_tag(p_add(lds[L_X0 + lr * kPH + u], hn), seq, xr, o_u, sA);  // x2 = x1 + h2
                    bst_tag(hn, seq, xr, o_u, sA + kPH * 8);
                } else {  // gh1 (r, z, n) of (row lr, unit u) for GRU1 at the end of this step
                    const float* b = lds + L_BIAS + (og - 16);  // b_hh1 of unit u
                    const u4v v = {__float_as_uint(p_add(s0, b[0])), __float_as_uint(p_add(s1, b[16])),
                                   __float_as_uint(p_add(s2, b[32])), 0u};
                    __builtin_amdgcn_raw_buffer_store_b128(
                        v, xr, (unsigned)((((t & 1) * kPNR + lr) * kPH + u) * 4) * 4u, XB_G * 4, 0);
                }
            }
            // this wave's reads of X0 (x1) are done (and its publishes issued): hop A may
            // overwrite X0 once all four GRU2 waves have arrived (x0_free below)
            if (!X2B && gate_a && (tid & 63) == 0)
                __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(lds) + L_ARR, 1u, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);  // (orders this wave's X0 reads before it)
        }
        __builtin_amdgcn_s_setprio(0);
        XSTAMP(30);
        PSTAMP(1);
        // ===== hop A: stage x2 -> X0, h2 -> XH2 (waves 0-3) ======================================
        // Late h2: hop A waits for x2 only; waves 0-3 fetch h2 (published with x2, needed first
        // by the off-path W_hh2 h2 of hop B) during stage B, where they are otherwise idle.
        // Local x2 (RAW): x1 is the same in every slot (GRU1 runs redundantly), so hop A carries
        // h2 only and each poll lane forms x2 = x1 + h2 of its couples itself -- the producer's
        // own fp32 add on the same operands (bit-identical x2), one publish instead of two, and
        // no second poll for h2. (Polling x2 with all 8 waves measured slower: 6.38 vs 6.28 us.)
        // X0 holds x1 until every GRU2 wave (0-3) has finished its stage-A products: a wave whose
        // hop-A poll completes early (its producer slots were ahead, e.g. at the launch's first
        // step) must not overwrite couples that a slower wave of this workgroup still reads
        // (the sparse instances' per-lane work differs between waves). Below kPNR rows per
        // group x2 goes to its own rows (L_X2) and nothing is waited for; at kPNR rows (no spare
        // row slots) it is formed in place after the arrival guard: waves 0-3 only, normally
        // satisfied on the first read.
        // (the counter is read once before the poll: when the four waves have arrived by then,
        // as they normally have, nothing is waited for after it)
        const unsigned arr_want = 4u * (unsigned)(t - a.t0 + 1);
        const bool arr_early = X2B || !wv_lo || __hip_atomic_load(reinterpret_cast<const unsigned*>(lds) + L_ARR,
                                                          __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= arr_want;
        auto x0_free = [&]() {
            const unsigned want = arr_want;
            const unsigned* arr = reinterpret_cast<const unsigned*>(lds) + L_ARR;
            if (arr_early) return;
            const unsigned t0s = p_now();
            while (__hip_atomic_load(arr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < want) {
                __builtin_amdgcn_s_sleep(1);
                if (p_now() - t0s > kSpinTicks) {  // (unreachable: every wave 0-3 arrives)
                    lds[L_FAIL] = 1.f;
                    break;
                }
            }
        };
        if (X2L) {
            if (wv_lo) {
                unsigned off[NR];
                float2* dst[NR];
#pragma unroll
                for (int m = 0; m < NR; ++m) {  // couple tl of row m: h2 -> XH2
                    off[m] = (unsigned)((m * 5 + 1) * kPH + 2 * tl) * 8u;
                    dst[m] = reinterpret_cast<float2*>(lds + L_XH2 + m * kPH) + tl;
                }
                if (!poll_couples<NR>(xr, off, sA, seq, dst, a.ctl)) lds[L_FAIL] = 1.f;
                x0_free();
#pragma unroll
                for (int m = 0; m < NR; ++m) {  // x2 = x1 + h2 of the same couples (own writes)
                    const float2* x = reinterpret_cast<const float2*>(lds + L_X0 + m * kPH) + tl;
                    float2* y = reinterpret_cast<float2*>(lds + (X2B ? L_X2 + m * kPNR * kPH : L_X0 + m * kPH)) + tl;
                    const float2 h = *dst[m];
                    float2 v = *x;
                    v.x = p_add(v.x, h.x);
                    v.y = p_add(v.y, h.y);
                    *y = v;
                }
            }
        } else if (wv_lo) {  // x2 -> X2 (X0 at kPNR rows), polling the tagged pairs, one pass
            unsigned off[NR];
            float2* dst[NR];
#pragma unroll
            for (int m = 0; m < NR; ++m) {  // couple tl of row m
                off[m] = (unsigned)(m * 5 * kPH + 2 * tl) * 8u;
                dst[m] = reinterpret_cast<float2*>(lds + (X2B ? L_X2 + m * kPNR * kPH : L_X0 + m * kPH)) + tl;
            }
            x0_free();  // (the poll writes X0 itself)
            if (!poll_couples<NR>(xr, off, sA, seq, dst, a.ctl)) lds[L_FAIL] = 1.f;
        }
        __syncthreads();
        PSTAMP(2);
        // fc1 / fc2: this thread's register rows wr[24..31] with the rows of Xs (row stride XS), relu
        auto mv1 = [&](float bias, const float4* Xs, auto xs_c) {
            constexpr int XS = decltype(xs_c)::value;
            constexpr int QB = NR >= 4 ? 1 : kPQB1;
            float s0 = 0.f;
            v2f acc[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r] = (v2f){0.f, 0.f};
            if constexpr (SP) {
                unsigned m[1] = {si.x >> 24}, p[1] = {si.z >> 16};
                v2f (&a1)[NR][1] = *reinterpret_cast<v2f(*)[NR][1]>(&acc);
                sp_products<NR, 1, 0xF, XS>(Wsp, Xs, m, p, kc, a1);
            } else
#pragma unroll
            for (int qb = 0; qb < 8; qb += QB) {
                __builtin_amdgcn_sched_barrier(0);
                float4 xq[NR][QB];
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int q = 0; q < QB; ++q) xq[r][q] = Xs[r * XS + 16 * (qb + q) + kc];
#pragma unroll
                for (int r = 0; r < NR; ++r)
#pragma unroll
                    for (int q = 0; q < QB; ++q) dot4(acc[r], wr[24 + qb + q], xq[r][q]);
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const float t0 = row16_sum(hsum(acc[r]));
                if (kc == r) s0 = t0;
            }
            const float y = p_add(s0, bias);
            return y > 0.f ? y : 0.f;
        };
        // ================= stage B: fc1 (waves 4-7, critical) ================================
        if (!gate_a) {
            const float y = mv1(pc0, X2, std::integral_constant<int, X2S>());
            // gh1 (hop A) must be in L2 before this wave's y1 can be seen
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (kc < NR) bst_tag(y, seq, xr, o_y, XB_B * 4);
        } else if (!X2L) {  // late h2 -> XH2 (tags stored with x2's: one pass)
            unsigned off[NR];
            float2* dst[NR];
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                off[m] = (unsigned)((m * 5 + 1) * kPH + 2 * tl) * 8u;
                dst[m] = reinterpret_cast<float2*>(lds + L_XH2 + m * kPH) + tl;
            }
            if (!poll_couples<NR>(xr, off, sA, seq, dst, a.ctl)) lds[L_FAIL] = 1.f;
        }
        // gh2 = W_hh2 h2 + b_hh2 (next step's GRU2), off the critical path, spread over the
        // exchange waits: rows r % 3 == 0 by waves 0-3 in hop B, r % 3 == 1 by waves 4-7 in hop
        // C, r % 3 == 2 by waves 4-7 in hop D (LDS weights, h2 staged in XH2)
        // window of row r's gh2: 0 hop B (waves 0-3), 1 hop C (waves 4-7), 2 hop D (waves 4-7)
        auto hh2_win = [](int r) { return r % 3; };
        auto hh2_rows = [&](auto win_c, int ul) {
            constexpr int WIN = decltype(win_c)::value;
            const float4* Wh = reinterpret_cast<const float4*>(lds + L_W) + (size_t)ul * 3 * kPK4;
            // weights read from LDS once per window, the window's rows accumulated per weight
            // load (each accumulator sums in the same k order as a per-row loop would)
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            v2f acc[NR][3];
#pragma unroll
            for (int r = 0; r < NR; ++r)
#pragma unroll
                for (int j = 0; j < 3; ++j) acc[r][j] = (v2f){0.f, 0.f};
            if constexpr (SP) {
                const unsigned mx = si.y, pb = si.w & 0xffffu;
                unsigned m[3] = {mx & 0xffu, (mx >> 8) & 0xffu, (mx >> 16) & 0xffu};
                const unsigned c0 = (unsigned)__builtin_popcount(m[0]), c1 = (unsigned)__builtin_popcount(m[1]);
                unsigned p[3] = {pb, pb + 16u * c0, pb + 16u * (c0 + c1)};
                sp_products<NR, 3, hh2_rowmask(WIN, NR)>(Wsp, XH2, m, p, kc, acc);
            } else
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                __builtin_amdgcn_sched_barrier(0);
                float4 w4[3];
#pragma unroll
                for (int j = 0; j < 3; ++j) w4[j] = Wh[j * kPK4 + 16 * q + kc];
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if (hh2_win(r) != WIN) continue;
                    const float4 x4 = XH2[r * kPK4 + 16 * q + kc];
#pragma unroll
                    for (int j = 0; j < 3; ++j) dot4(acc[r][j], w4[j], x4);
                }
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                if (hh2_win(r) != WIN) continue;
                const float t0 = row16_sum(hsum(acc[r][0]));
                const float t1 = row16_sum(hsum(acc[r][1]));
                const float t2 = row16_sum(hsum(acc[r][2]));
                if (kc == r) {
                    s0 = t0;
                    s1 = t1;
                    s2 = t2;
                }
            }
            if (kc < NR && hh2_win(kc) == WIN) {
                float* gh2 = lds + L_GH2 + ul * 3 * kPNR + kc;
                const float* b = lds + L_BIAS + 48 + ul;  // b_hh2 of unit 16 w + ul
                gh2[0] = p_add(s0, b[0]);
                gh2[kPNR] = p_add(s1, b[16]);
                gh2[2 * kPNR] = p_add(s2, b[32]);
            }
        };
        PSTAMP(3);
        __syncthreads();  // fc1 has read X0: y1 may be staged over it
        // ===== hop B: stage y1 -> X0 (waves 4-7) | W_hh2 h2 rows r % 3 == 0 (waves 0-3) =======
        if (!wv_lo) {
            unsigned off[NR];
            float2* dst[NR];
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                off[m] = (unsigned)(m * kPH + 2 * tl) * 8u;
                dst[m] = reinterpret_cast<float2*>(lds + L_X0 + m * kPH) + tl;
            }
            if (!poll_couples<NR>(xr, off, XB_B * 4, seq, dst, a.ctl)) lds[L_FAIL] = 1.f;
        } else {
            hh2_rows(std::integral_constant<int, 0>(), og);
            XSTAMP(31);
        }
        __syncthreads();
        PSTAMP(4);
        // ================= stage C: fc2 (waves 0-3, critical) ================================
        if (gate_a) {
            const float y = mv1(pf2, X0, std::integral_constant<int, kPK4>());
            if (kc < NR) bst_tag(y, seq, xr, o_y, XB_C * 4);
        } else {
            // P1 ring: operands of P1(t + 2), issued while no poll is in flight on this CU
            // (fc2 is LDS + VALU on waves 0-3); stored in hop C
            p1_loads(t + 2);
        }
        PSTAMP(5);
        __syncthreads();  // fc2 has read X0: y2 may be staged over it
        // ===== hop C: stage y2 -> X0 (waves 0-3) | W_hh2 h2 rows r % 3 == 1 (waves 4-7) =======
        if (wv_lo) {
            unsigned off[NR];
            float2* dst[NR];
#pragma unroll
            for (int m = 0; m < NR; ++m) {
                off[m] = (unsigned)(m * kPH + 2 * tl) * 8u;
                dst[m] = reinterpret_cast<float2*>(lds + L_X0 + m * kPH) + tl;
            }
            if (!poll_couples<NR>(xr, off, XB_C * 4, seq, dst, a.ctl)) lds[L_FAIL] = 1.f;
        } else {
            // P1 ring: P1(t + 2) (operands loaded in stage C) into slot t & 1 (P1(t) there was
            // read at step t - 1: every slot is past it)
            if (NR > 1) hh2_rows(std::integral_constant<int, 1>(), og - 16);
            p1_store(t + 2);
        }
        __syncthreads();
        PSTAMP(6);
        float pG[NR][3];  // GRU1 operands, loaded once this wave's fc3 work is issued
        auto gru1_loads = [&]() {
            // gh1 (stage A) was drained by its producer waves before they stored y1 (stage B),
            // and this workgroup has seen every slot's y1 tag (stage C staging): plain loads
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const u4v v = __builtin_amdgcn_raw_buffer_load_b128(
                    xr, o_tid * 4u, (unsigned)(XB_G + ((t & 1) * kPNR + r) * kPH * 4) * 4u, kCpNT);
                pG[r][0] = __uint_as_float(v.x);
                pG[r][1] = __uint_as_float(v.y);
                pG[r][2] = __uint_as_float(v.z);
            }
            if constexpr (P1R)  // P1(t + 1) from the ring (stored at step t - 1 / the prologue,
                                // ordered before this step's y1 as gh1 is)
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const u4v v = __builtin_amdgcn_raw_buffer_load_b128(
                        xr, o_tid * 4u, (unsigned)(XB_P + (((t + 1) & 1) * kPNR + r) * kPH * 4) * 4u, kCpNT);
                    pP[r][0] = __uint_as_float(v.x);
                    pP[r][1] = __uint_as_float(v.y);
                    pP[r][2] = __uint_as_float(v.z);
                    pC[r] = __uint_as_float(v.w);
                }
            prefetch(t, t + 1);  // pgn, not pgum: the fc3 epilogue still reads pgum
        };

        const int st = EARLY ? tid - 256 : tid;
        {
            float s0 = 0.f;
            auto fc3 = [&]() {
                if (!has_cls) return;
                const float4* Wf = reinterpret_cast<const float4*>(lds + L_FC3) + (size_t)og * kPK4;
                v2f acc[NR];
#pragma unroll
                for (int r = 0; r < NR; ++r) acc[r] = (v2f){0.f, 0.f};
                if constexpr (SP) {
                    unsigned m[1] = {si.y >> 24}, p[1] = {si.w >> 16};
                    v2f (&a1)[NR][1] = *reinterpret_cast<v2f(*)[NR][1]>(&acc);
                    sp_products<NR, 1>(Wsp, X0, m, p, kc, a1);
                } else
#pragma unroll
                for (int qb = 0; qb < 8; qb += 4) {
                    __builtin_amdgcn_sched_barrier(0);
                    float4 wq[4];  // fc3 weights: one LDS read per step (10-bit: registers)
#pragma unroll
                    for (int q = 0; q < 4; ++q) wq[q] = FC3R && !SP ? wr[(32 + qb + q) % NW] : Wf[16 * (qb + q) + kc];
#pragma unroll
                    for (int r = 0; r < NR; ++r) {
                        float4 xq[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) xq[q] = X0[r * kPK4 + 16 * (qb + q) + kc];
#pragma unroll
                        for (int q = 0; q < 4; ++q) dot4(acc[r], wq[q], xq[q]);
                    }
                }
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const float t0 = row16_sum(hsum(acc[r]));
                    if (kc == r) s0 = t0;
                }
            };
            // (separate paths, so the GRU1 operands of waves 4-7 hold no register during fc3)
            if (EARLY) {
                if (wv_lo) {
                    fc3();
                    XSTAMP(26);
                } else {
                    gru1_loads();
                }
            } else {
                fc3();
            }
            float* red = lds + L_RED;
            // [og][r] (logit, noise word) of (row r, class og's); wave 0 forms the candidate keys
            // (cand_key) as it reduces them
            if (kc < NR) {
                float l = -INFINITY;
                if (has_cls) {
                    l = p_add(s0, lds[L_BCLS + og]);
                    p_dbg_logit<DBG>(a.dbg, t + lvm.y, lrow, cls, a.B, a.n_classes, l);
                    if (MOL)  // MOL: logit (row kc, class cls) as a tagged pair, polled directly
                        bst_tag(l, seq, xr, (unsigned)(kc * 32 + cls) * 8u, (XB_D + XB_D_LOG) * 4);
                }
                *reinterpret_cast<float2*>(red + (og * kPNR + kc) * 2) = make_float2(l, pgum);
            }
            XSTAMP(28);
            __syncthreads();
            PSTAMP(11);
            if (wv_lo) {
            if (wave == 0) {
                if (!MOL) {
                    // slot candidate per row: the max key, tagged with the step (no flag, no wait)
                    const unsigned tag = key_tag(seq);
                    int tt = tid;  // (lane offsets recomputed per step: hoisted ones cost registers)
                    asm volatile("" : "+v"(tt));
                    if (a.cpw <= 16) {  // DPP row r = lane / 16 reduces the slot's classes of row r
                        const int r = tt >> 4, o = tt & 15;
                        uint32_t bh = 0, bl = 0;
                        if (r < NR && o < a.cpw && a.cpw * w + o < a.n_classes) {
                            const float2 lg = *reinterpret_cast<const float2*>(red + (o * kPNR + r) * 2);
                            const CandKey k = cand_key(lg.x, __float_as_uint(lg.y), a.cpw * w + o);
                            bh = k.hi;
                            bl = k.lo;
                        }
                        row16_kmax(bh, bl);
                        const int rr = r;
                        if (r < NR && o == 0)
                            __builtin_amdgcn_raw_buffer_store_b64((u2v){bh, bl | tag}, xr,
                                                                  (unsigned)((w * kPNR + rr) * 2) * 4u, XB_D * 4, 0);
                    } else {
#pragma unroll
                        for (int rb = 0; rb < NR; rb += 2) {
                            const int r = rb + (tt >> 5), o = tt & 31;
                            uint32_t bh = 0, bl = 0;
                            if (r < NR && o < a.cpw && a.cpw * w + o < a.n_classes) {
                                const float2 lg = *reinterpret_cast<const float2*>(red + (o * kPNR + r) * 2);
                                const CandKey k = cand_key(lg.x, __float_as_uint(lg.y), a.cpw * w + o);
                                bh = k.hi;
                                bl = k.lo;
                            }
                            half_kmax(bh, bl);
                            const int rr = r;
                            if (r < NR && o == 31)
                                __builtin_amdgcn_raw_buffer_store_b64((u2v){bh, bl | tag}, xr,
                                                                      (unsigned)((w * kPNR + rr) * 2) * 4u, XB_D * 4, 0);
                        }
                    }
                }
            }
            if (EARLY) {  // waves 0-3: GRU1 operands after the candidate publish
                gru1_loads();
                XSTAMP(27);
            }
            } else {
                // hop D: W_hh2 h2 rows r % 3 == 2 (waves 4-7, before their candidate poll)
                if (NR > 2) hh2_rows(std::integral_constant<int, 2>(), og - 16);
            }
        }
        if (FC3R) gru1_loads();
        PSTAMP(7);
        PSTAMP(8);
        // ================= sample of step t (redundant in every workgroup) ==================
        if (!MOL) {
            if (st >= 0 && st < 32 * NR) {  // half-wave r: lane o polls slot o's candidate of row r
                const int r = st >> 5, o = st & 31;
                const unsigned want = key_tag(seq);
                const unsigned t0 = p_now();
                unsigned n = 0;
                uint32_t bh, bl;
                {
                    const unsigned off = (unsigned)((o * kPNR + r) * 2) * 4u;
                    u2v c = __builtin_amdgcn_raw_buffer_load_b64(xr, off, XB_D * 4, kCpNT);
                    while (true) {  // two polls in flight (see poll_couples)
                        const u2v c1 = __builtin_amdgcn_raw_buffer_load_b64(xr, off, XB_D * 4, kCpNT);
                        if (__all((c.y & kKeyTagMask) == want)) break;
                        c = c1;
                        if ((++n & 255) == 0) {
                            if (ld_sc1_u(a.ctl + PC_ERR) || p_now() - t0 > kSpinTicks) {
                                if ((tid & 63) == 0) atomicMax(a.ctl + PC_ERR, 2u);
                                lds[L_FAIL] = 1.f;
                                break;
                            }
                        }
                    }
                    bh = c.x;
                    bl = c.y;
                }
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
                        int rr = r;  // (recomputed per step: a hoisted offset costs a register)
                        asm volatile("" : "+v"(rr));
                        const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[rr];
                        const unsigned ro = (unsigned)(vm.x * a.ld + vm.y);
                        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)bi, mk_rsrc(a.labels),
                                                              ro * 2u, (unsigned)t * 2u, 0);
                        bst(xv, mk_rsrc(a.samples), ro * 4u, (unsigned)t * 4u);
                    }
                }
            }
        } else if (st >= 0 && st < 32 * NR) {
            // MOL: vocoder/distribution.py:104-140. Half-wave r: lane k polls logit k of row r
            // (tagged pair) and holds draw k of k_mol_noise (gm_k = log(-log(u1_k)), k < 10;
            // gm_10 = log(u2) - log(1 - u2)), prefetched a step ahead
            const int r = st >> 5, k = st & 31;
            const unsigned off = (unsigned)((r * 32 + k) * 2) * 4u;
            const unsigned so = (XB_D + XB_D_LOG) * 4;
            const bool real = k < a.n_classes;
            const unsigned t0 = p_now();
            unsigned n = 0;
            u2v c = __builtin_amdgcn_raw_buffer_load_b64(xr, off, so, kCpNT);
            while (true) {  // two polls in flight (see poll_couples)
                const u2v c1 = __builtin_amdgcn_raw_buffer_load_b64(xr, off, so, kCpNT);
                if (__all(!real || c.y == seq)) break;
                c = c1;
                if ((++n & 255) == 0) {
                    if (ld_sc1_u(a.ctl + PC_ERR) || p_now() - t0 > kSpinTicks) {
                        if ((tid & 63) == 0) atomicMax(a.ctl + PC_ERR, 2u);
                        lds[L_FAIL] = 1.f;
                        break;
                    }
                }
            }
            const float lk = __uint_as_float(c.x);
            float bv;
            {
#pragma clang fp contract(off)
                bv = k < 10 ? lk - pgum : -INFINITY;
            }
            int bi = k < 10 ? k : 0x7fffffff;
            row16_argmax(bv, bi);  // first max over k < 10 (lanes 0-15 of the half)
            const int base = (tid & 63) & 32;
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
                    int rr = r;
                    asm volatile("" : "+v"(rr));
                    const int2 vm = reinterpret_cast<const int2*>(lds + L_VM)[rr];
                    bst(xv, mk_rsrc(a.samples), (unsigned)(vm.x * a.ld + vm.y) * 4u, (unsigned)t * 4u);
                }
            }
        }
        __syncthreads();
        // The step's one failure check: a wave whose poll gave up (timeout, or PC_ERR raised by
        // another slot) finishes the step on whatever its buffers hold, and every other poll
        // of the step ends within 256 spins of PC_ERR, so all waves reach this barrier. (A check
        // after every hop's barrier cost an LDS round trip each, in front of the stage's own
        // LDS reads.)
        if (lds[L_FAIL] != 0.f) return;
        PSTAMP(9);
        // (at the last step this GRU1 runs on clamped inputs and its result goes unused)
        // ================= GRU1 of step t+1 for all 512 units (redundant) ===================
        //   gi = W_ih1 (cI + w0 x) + b_ih1 = P1 + v x ; x1 = (cI + w0 x) + h1
        const float w0j = lds[L_W0 + tid];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const float x = lds[L_SX + r];
            const float hn = p_gru(fmaf(vj0, x, pP[r][0]), fmaf(vj1, x, pP[r][1]),
                                   fmaf(vj2, x, pP[r][2]), pG[r][0], pG[r][1], pG[r][2], h1[r]);
            h1[r] = hn;
            lds[L_X0 + r * kPH + tid] = p_add(fmaf(w0j, x, pC[r]), hn);
            lds[L_X1 + r * kPH + tid] = hn;
        }
        pgum = pgn;
        if (w == 0 && tid == 0) {
            // (rotated: the launch's share of the call, steps scaled to S per launch)
            if (g == 0) p_progress(a.progress, a.prog_base, ROT ? (int)((long long)t * a.S / t1g) : t, t);
            if (p_abort(a.ctl, a.progress, t)) lds[L_FAIL] = 1.f;  // seen after the next sample
        }
        __syncthreads();
        PSTAMP(10);
    }
#undef PSTAMP
#undef XSTAMP
    if (a.stamps && g == 0 && w == 0 && tid == 0) a.stamps[1] = p_now();
    // ---- save the chunk state --------------------------------------------------------------
    // (addresses recomputed here: values kept alive across the step loop cost registers)
    if (ROT || a.t1 < a.S) {
        int tx = tid;
        asm volatile("" : "+v"(tx));
        const int kx = tx & 15, ux = 16 * w + ((tx >> 4) & 15), rx = vmap_g(kx < NR ? kx : 0).x;
        if (w == 0)
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int row = vmap_g(r).x;
                a.st_x1[(size_t)row * H + tx] = lds[L_X0 + r * kPH + tx];
                a.st_h1[(size_t)row * H + tx] = lds[L_X1 + r * kPH + tx];
            }
        if (own) {
            a.st_h2[(size_t)rx * H + ux] = h2r;
#pragma unroll
            for (int j = 0; j < 3; ++j)
                a.st_gh2[(size_t)rx * 3 * H + j * H + ux] = lds[L_GH2 + (og * 3 + j) * kPNR + kc];
        }
    }
}

template <int NR, bool FC3R, bool MOL, bool P1R, bool ROT, bool DBG, bool SP = false>
__global__ __launch_bounds__(kPT, 1) void k_persist(PersistArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    __shared__ int s_group, s_slot, s_ok;
    // ---- group formation (placement-independent: a group is whatever shares an XCD) ----
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
    if constexpr (ROT && NR > 1) {
        // a rotated launch holds groups of NR and of NR - 1 rows: each runs its own body
        if (__builtin_amdgcn_readfirstlane(a.gnr[g]) == NR)
            persist_body<NR, FC3R, MOL, P1R, true, DBG, SP>(a, lds, g, w);
        else
            persist_body<NR - 1, FC3R, MOL, P1R, true, DBG, SP>(a, lds, g, w);
    } else {
        persist_body<NR, FC3R, MOL, P1R, ROT, DBG, SP>(a, lds, g, w);
    }
}

#if WRNN_PERSIST_PART != 2
// Step-0 state: GRU1 with x = 0, h = 0, gh = b_hh1 -> x1(0), h1(0); h2 = 0, gh2 = b_hh2.
__global__ __launch_bounds__(kPT) void k_persist_init(PersistArgs a) {
    const int row = blockIdx.x, j = threadIdx.x, H = kPH;
    const float* P1 = a.P1 + ((size_t)row * H + j) * 4;  // step 0: (r, z, n, cI) of unit j
    const float hn = p_gru(P1[0], P1[1], P1[2], a.b_hh1[j], a.b_hh1[H + j], a.b_hh1[2 * H + j], 0.f);
    a.st_h1[(size_t)row * H + j] = hn;
    a.st_x1[(size_t)row * H + j] = p_add(P1[3], hn);
    a.st_h2[(size_t)row * H + j] = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) a.st_gh2[(size_t)row * 3 * H + k * H + j] = a.b_hh2[k * H + j];
}

hipError_t launch_persist_init(const PersistArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_persist_init, dim3(a.B), dim3(kPT), 0, s, a);
    return hipGetLastError();
}

// RAW Gumbel noise of every (step, row, class) of rows [r0, r0 + nrows) of the [S][ld][n]
// buffer in the fixed-point form philox.h gumbel_q_of (wide launches form theirs in-kernel, so
// a plan with them fills only the register-resident launches' rows)
__global__ __launch_bounds__(256) void k_gumbel(uint4* g, int S, int r0, int nrows, int ld, int ng,
                                                const RowInfo* rows, uint32_t k0, uint32_t k1) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // (t, r, k4)
    const size_t total = (size_t)S * nrows * ng;
    if (i >= total) return;
    const int k4 = (int)(i % ng);
    const size_t tr = i / ng;
    const int r = r0 + (int)(tr % nrows), t = (int)(tr / nrows);
    const RowInfo ri = rows[r];
    const U4 o = philox4x32_10((uint32_t)k4, (uint32_t)t, (uint32_t)ri.fold, ri.stream, k0, k1);
    g[((size_t)t * ld + r) * ng + k4] = make_uint4(gumbel_q_of(o.x), gumbel_q_of(o.y), gumbel_q_of(o.z), gumbel_q_of(o.w));
}

hipError_t launch_gumbel(float* g, int S, int nrows, int n_classes, const RowInfo* rows,
                         uint32_t k0, uint32_t k1, hipStream_t s) {
    return launch_gumbel_rows(g, S, 0, nrows, nrows, n_classes, rows, k0, k1, s);
}

hipError_t launch_gumbel_rows(float* g, int S, int r0, int nrows, int ld, int n_classes,
                              const RowInfo* rows, uint32_t k0, uint32_t k1, hipStream_t s) {
    if (n_classes % 4 || r0 < 0 || r0 + nrows > ld) return hipErrorInvalidValue;
    const int ng = n_classes / 4;
    const size_t total = (size_t)S * nrows * ng;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gumbel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<uint4*>(g), S, r0, nrows, ld, ng, rows, k0, k1);
    return hipGetLastError();
}

// MOL noise of the RNG contract (philox.h, oracle/philox.py mol_uniforms) in the form the
// sampler consumes, with the sampler's own float operations (kernels_step.hip k_sample):
// [k < 10] = log(-log(u1_k)), [10] = log(u2) - log(1 - u2), [11] = 0.
__global__ __launch_bounds__(256) void k_mol_noise(float* out, int S, int nrows, const RowInfo* rows,
                                                   uint32_t k0, uint32_t k1) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;  // (t, r)
    if (i >= (size_t)S * nrows) return;
    const int r = (int)(i % nrows), t = (int)(i / nrows);
    const RowInfo ri = rows[r];
    uint32_t wd[12];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const U4 o = philox4x32_10(kMolDomain | (uint32_t)j, (uint32_t)t, (uint32_t)ri.fold, ri.stream, k0, k1);
        wd[4 * j] = o.x;
        wd[4 * j + 1] = o.y;
        wd[4 * j + 2] = o.z;
        wd[4 * j + 3] = o.w;
    }
    float* d = out + i * kMolNoise;
    {
#pragma clang fp contract(off)
        for (int k = 0; k < 10; ++k) d[k] = logf(-logf(mol_uniform_from_u32(wd[k])));
        const float u2 = mol_uniform_from_u32(wd[10]);
        d[10] = logf(u2) - logf(1.0f - u2);
        d[11] = 0.f;
    }
}

hipError_t launch_mol_noise(float* out, int S, int nrows, const RowInfo* rows, uint32_t k0,
                            uint32_t k1, hipStream_t s) {
    const size_t total = (size_t)S * nrows;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mol_noise, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, out, S,
                       nrows, rows, k0, k1);
    return hipGetLastError();
}

size_t persist_lds_bytes() { return (size_t)L_TOTAL * sizeof(float); }
size_t persist_xbuf_floats() { return (size_t)kPG * XB_GROUP; }
#endif  // WRNN_PERSIST_PART != 2

template <int NR, bool FC3R, bool MOL, bool P1R>
hipError_t launch_persist_t(const PersistArgs& a, hipStream_t s) {
    if constexpr (P1R) {  // sparse instances (a.sparse: the pruned-weight image), ring only
        if (a.sparse) {
            if constexpr (!FC3R && NR >= 2)
                if (a.vmap) {
                    if (a.dbg.out) return persist_launch<k_persist<NR, FC3R, MOL, P1R, true, true, true>>(persist_lds_bytes(), a, s);
                    return persist_launch<k_persist<NR, FC3R, MOL, P1R, true, false, true>>(persist_lds_bytes(), a, s);
                }
            if (a.vmap) return hipErrorInvalidValue;
            if (a.dbg.out) return persist_launch<k_persist<NR, FC3R, MOL, P1R, false, true, true>>(persist_lds_bytes(), a, s);
            return persist_launch<k_persist<NR, FC3R, MOL, P1R, false, false, true>>(persist_lds_bytes(), a, s);
        }
    }
    if (a.sparse) return hipErrorInvalidValue;
    if constexpr (P1R && !FC3R && NR >= 2) {  // rotated launches (a.vmap): 9-bit ring variants
        if (a.vmap) {
            if (a.dbg.out) return persist_launch<k_persist<NR, FC3R, MOL, P1R, true, true>>(persist_lds_bytes(), a, s);
            return persist_launch<k_persist<NR, FC3R, MOL, P1R, true, false>>(persist_lds_bytes(), a, s);
        }
    }
    if (a.vmap) return hipErrorInvalidValue;
    if (a.dbg.out) return persist_launch<k_persist<NR, FC3R, MOL, P1R, false, true>>(persist_lds_bytes(), a, s);
    return persist_launch<k_persist<NR, FC3R, MOL, P1R, false, false>>(persist_lds_bytes(), a, s);
}

template <int NR, bool FC3R, bool MOL, bool P1R, bool SP = false>
int persist_spill_t() {
    if constexpr (SP && !P1R) {
        return -1;
    } else {
        hipFuncAttributes fa;
        if (hipFuncGetAttributes(&fa, (const void*)k_persist<NR, FC3R, MOL, P1R, false, false, SP>) != hipSuccess) return -1;
        return (int)fa.localSizeBytes;
    }
}

// scratch bytes of the rotated instance (groups of NR and NR - 1 rows); -1 when none exists
template <int NR, bool MOL, bool SP = false>
int persist_rot_spill_t() {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)k_persist<NR, false, MOL, true, true, false, SP>) != hipSuccess) return -1;
    return (int)fa.localSizeBytes;
}

#if WRNN_PERSIST_PART != 1
int persist_rot_scratch_mol(int nr, int sparse) {
    switch (nr * 2 + (sparse ? 1 : 0)) {
        case 4: return persist_rot_spill_t<2, true>();
        case 5: return persist_rot_spill_t<2, true, true>();
        case 6: return persist_rot_spill_t<3, true>();
        case 7: return persist_rot_spill_t<3, true, true>();
        case 8: return persist_rot_spill_t<4, true>();
        case 9: return persist_rot_spill_t<4, true, true>();
        default: return -1;
    }
}
#else
int persist_rot_scratch_mol(int nr, int sparse);
#endif

#if WRNN_PERSIST_PART != 2
// Scratch bytes of the rotated instance with groups of nr and nr - 1 rows (9-bit RAW or MOL,
// P1 ring); -1 when none exists.
int persist_rot_scratch(int nr, int mode, int sparse) {
    if (mode != 0) return persist_rot_scratch_mol(nr, sparse);
    switch (nr * 2 + (sparse ? 1 : 0)) {
        case 4: return persist_rot_spill_t<2, false>();
        case 5: return persist_rot_spill_t<2, false, true>();
        case 6: return persist_rot_spill_t<3, false>();
        case 7: return persist_rot_spill_t<3, false, true>();
        case 8: return persist_rot_spill_t<4, false>();
        case 9: return persist_rot_spill_t<4, false, true>();
        default: return -1;
    }
}
#endif

#if WRNN_PERSIST_PART != 1
// MOL variants (30 classes: cpw <= 16)
int persist_spill_mol(int nr, int ring, int sparse) {
    if (sparse) {
        switch (nr) {
            case 1: return persist_spill_t<1, false, true, true, true>();
            case 2: return persist_spill_t<2, false, true, true, true>();
            case 3: return persist_spill_t<3, false, true, true, true>();
            case 4: return persist_spill_t<4, false, true, true, true>();
            default: return -1;
        }
    }
    switch (nr * 2 + (ring ? 1 : 0)) {
        case 2: return persist_spill_t<1, false, true, false>();
        case 3: return persist_spill_t<1, false, true, true>();
        case 4: return persist_spill_t<2, false, true, false>();
        case 5: return persist_spill_t<2, false, true, true>();
        case 6: return persist_spill_t<3, false, true, false>();
        case 7: return persist_spill_t<3, false, true, true>();
        case 8: return persist_spill_t<4, false, true, false>();
        case 9: return persist_spill_t<4, false, true, true>();
        default: return -1;
    }
}

hipError_t launch_persist_mol(const PersistArgs& a, hipStream_t s) {
    const bool ring = a.p1q != nullptr;
    switch (a.nr * 2 + (ring ? 1 : 0)) {
        case 2: return launch_persist_t<1, false, true, false>(a, s);
        case 3: return launch_persist_t<1, false, true, true>(a, s);
        case 4: return launch_persist_t<2, false, true, false>(a, s);
        case 5: return launch_persist_t<2, false, true, true>(a, s);
        case 6: return launch_persist_t<3, false, true, false>(a, s);
        case 7: return launch_persist_t<3, false, true, true>(a, s);
        case 8: return launch_persist_t<4, false, true, false>(a, s);
        case 9: return launch_persist_t<4, false, true, true>(a, s);
        default: return hipErrorInvalidValue;
    }
}
#else
int persist_spill_mol(int nr, int ring, int sparse);
hipError_t launch_persist_mol(const PersistArgs& a, hipStream_t s);
#endif

#if WRNN_PERSIST_PART != 2
template <int NR, bool P1R>
int persist_spill_nr(int cpw, int mode, int sparse) {
    if (mode != 0) return cpw <= 16 ? persist_spill_mol(NR, P1R, sparse) : -1;  // MOL: 30 classes
    if (sparse)
        return !P1R ? -1 : cpw > 16 ? persist_spill_t<NR, true, false, P1R, true>()
                                    : persist_spill_t<NR, false, false, P1R, true>();
    return cpw > 16 ? persist_spill_t<NR, true, false, P1R>() : persist_spill_t<NR, false, false, P1R>();
}

// Scratch bytes of the (rows per group, classes per slot, mode, P1 ring, sparse) variant; -1
// when it does not exist (sparse instances: P1 ring only).
int persist_variant_scratch(int nr, int cpw, int mode, int ring, int sparse) {
    if (cpw < 1 || cpw > kPCls) return -1;
    switch (nr * 2 + (ring ? 1 : 0)) {
        case 2: return persist_spill_nr<1, false>(cpw, mode, sparse);
        case 3: return persist_spill_nr<1, true>(cpw, mode, sparse);
        case 4: return persist_spill_nr<2, false>(cpw, mode, sparse);
        case 5: return persist_spill_nr<2, true>(cpw, mode, sparse);
        case 6: return persist_spill_nr<3, false>(cpw, mode, sparse);
        case 7: return persist_spill_nr<3, true>(cpw, mode, sparse);
        case 8: return persist_spill_nr<4, false>(cpw, mode, sparse);
        case 9: return persist_spill_nr<4, true>(cpw, mode, sparse);
        default: return -1;
    }
}

// 1 when the variant exists and keeps its state in registers (no scratch spills: scratch
// traffic would serialise behind every exchange).
int persist_variant_ok(int nr, int cpw, int mode, int ring) {
    return persist_variant_scratch(nr, cpw, mode, ring, 0) == 0 ? 1 : 0;
}

template <int NR, bool P1R>
hipError_t launch_persist_nr(const PersistArgs& a, hipStream_t s) {
    if (a.mode != 0) return a.cpw <= 16 ? launch_persist_mol(a, s) : hipErrorInvalidValue;
    return a.cpw > 16 ? launch_persist_t<NR, true, false, P1R>(a, s) : launch_persist_t<NR, false, false, P1R>(a, s);
}

hipError_t launch_persist(const PersistArgs& a, hipStream_t s) {
    if (a.rb < 0 || a.nr < 1 || a.rb + kPG * a.nr > a.B || a.cpw < 1 || a.cpw > kPCls || a.cpw * kPM < a.n_classes)
        return hipErrorInvalidValue;
    const bool ring = a.p1q != nullptr;
    if (ring && (!a.p1a || !a.p1taps || a.hop <= 0)) return hipErrorInvalidValue;
    switch (a.nr * 2 + (ring ? 1 : 0)) {
        case 2: return launch_persist_nr<1, false>(a, s);
        case 3: return launch_persist_nr<1, true>(a, s);
        case 4: return launch_persist_nr<2, false>(a, s);
        case 5: return launch_persist_nr<2, true>(a, s);
        case 6: return launch_persist_nr<3, false>(a, s);
        case 7: return launch_persist_nr<3, true>(a, s);
        case 8: return launch_persist_nr<4, false>(a, s);
        case 9: return launch_persist_nr<4, true>(a, s);
        default: return hipErrorInvalidValue;
    }
}
#endif  // WRNN_PERSIST_PART != 2

}  // namespace wrnn
