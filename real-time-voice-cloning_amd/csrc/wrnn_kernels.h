// Internal declarations shared by the HIP kernels (kernels_*.hip) and the runtime
// (runtime.hip). Not part of the public ABI (include/wavernn_mi355x.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wrnn {

constexpr int kThreads = 256;  // every kernel: 4 wave64 per workgroup

// ---------------------------------------------------------------------------------------
// Recurrent step ("stage") kernels. One launch = up to 3 matvec segments that are
// independent of each other (a critical-path layer plus off-path recurrent products).
// ---------------------------------------------------------------------------------------
enum EpiKind : int {
    EPI_GRU = 0,        // torch GRUCell gates -> h (in place) and x_out = x_in + h
    EPI_BIAS3 = 1,      // out[r][g*H + j] = acc + bias  (W_hh h + b_hh ; W_ih1 cI + b_ih1)
    EPI_COND = 2,       // out[r][o] = acc + cond(frame)[o]
    EPI_COND_RELU = 3,  // out[r][o] = relu(acc + cond(frame)[o])
};

// Tile shapes (256 threads = NOG output groups x NRG row groups x KC k-chunks):
//   TILE_GATE: OPL 3 = the r,z,n gates of one unit per thread, NOG 4 units per tile
//   TILE_OUT : OPL 1 output per thread, NOG 4 outputs per tile
// NRG (1, 2 or 4) is a launch-wide template parameter chosen by the runtime.
enum TileCfg : int {
    TILE_GATE = 0,
    TILE_OUT = 1,
};
constexpr int kTileNOG = 4;
inline int tile_opl(int cfg) { return cfg == TILE_GATE ? 3 : 1; }

struct RowInfo {
    int pos0;        // global index of this row's step-0 position in per-position buffers
    int rel0;        // fold start inside its utterance: fold * (target + overlap)
    int L;           // valid upsampled length of its utterance (positions >= L are pad)
    int fbase;       // per-frame buffers: frame slot of the utterance's zero frame
    int fold;        // fold index inside its utterance (Philox counter word 2)
    uint32_t stream; // Philox counter word 3 of its utterance
};

struct Seg {
    const float* W;  // packed tiles, see pack_segment() in runtime.hip
    int n_out, n_tiles, kind, cfg;
    // input row r: X + x_off + r * x_ld + rows[r].pos0 * x_pld
    const float* X;
    long long x_off;
    int x_ld, x_pld;
    // outputs
    float* Y;
    int y_ld;
    const float* cond;  // row r: cond + frame(r) * c_ld   (c_ld == 0: one shared vector)
    int c_ld;
    const float* gh;    // EPI_GRU: W_hh h_prev + b_hh, [r][3H] gate-major
    float* h;           // EPI_GRU: hidden state [r][H], updated in place
    float* xout;        // EPI_GRU: x_in + h_new, [r][H]
    int H;
};

struct StageArgs {
    Seg seg[3];
    int nseg;
    int tile_start[4];  // blockIdx.x ranges per segment
    int nrows;
    int t;              // step index (selects frames of the conditioning)
    int hop;
    const RowInfo* rows;
    uint32_t* stamps;   // optional: workgroup w stores [2w] = start, [2w+1] = end
                        // (low 32 bits of s_memrealtime, 100 MHz) -- no atomics
    uint32_t* phases;   // optional diagnostic: workgroup w stores 6 stamps at [8w + i]
};

constexpr int kMaxStampWG = 2048;  // workgroups recorded per timed launch
constexpr int kStampEvery = 8;     // timed steps: t % kStampEvery == 0

// Logit capture for the teacher-forced gate (wrnn_set_debug_steps / wrnn_debug_logits): the
// pre-sampling logits (last linear layer + bias, before softmax / noise) of every row at up to
// kDbgSteps chosen steps. Off (out == nullptr) in production: one uniform branch per step.
constexpr int kDbgSteps = 8;
struct DbgLogits {
    float* out;             // [kDbgSteps][B][n_classes]
    const int* map;         // [S]: slot of step t in `out`, or -1
};

struct SampleArgs {
    int t;          // step whose logits are sampled; -1 = initial GRU1 only (x = 0)
    int S, nrows, n_classes, mode, H;
    const float* logits;   // [r][n_classes]
    const float* noise;    // RAW: [t][r][n_classes] Exp(1) variates
    float* samples;        // [r][S]
    int16_t* labels;       // [r][S] (RAW)
    int do_gru;            // compute GRU1 of step t+1
    const float* P1;       // [r][3H] = W_ih1 cI(t+1) + b_ih1
    const float* v;        // [3H]    = W_ih1 . I.weight[:,0]
    const float* gh1;      // [r][3H] = W_hh1 h1 + b_hh1
    float* h1;             // [r][H] in/out
    float* x1;             // [r][H] out: xI + h1
    const float* cI;       // folded [t][r][H]: I.weight[:,1:] . [m, a1[:31]] + I.bias
    const float* w0;       // [H] = I.weight[:, 0]
    const RowInfo* rows;
    uint32_t k0, k1;       // Philox key (MOL draws in-kernel)
    uint32_t* phases;      // optional diagnostic: workgroup w stores 6 stamps at [8w + i]
    DbgLogits dbg;         // rows indexed as in `logits` (the call's row space)
};

// ---------------------------------------------------------------------------------------
// GEMM-shaped precompute (upsample convs + conditioning), fp32 MFMA 32x32x2.
// D[m][n] = sum_k A(m,k) * B(k,n), epilogue per element.
// ---------------------------------------------------------------------------------------
struct GemmA {  // A(m, k)
    int kind;   // 0: row-major W[m*ld + k]; 1: cond-A (mel/aux gather for cI); 2: frame-A
    const float* p;
    int ld;
    // kind 1: row m = (fold f = m / S, step t = m % S), S = M / Bu -> position p = f * tpo + t;
    // mel_up channel-major [n_mel][ldm] + R channel-major [C][T]
    const float* mel;
    int ldm, n_mel, L, hop;
    const float* R;
    int ldr, r_off, n_aux;
    int Bu, tpo;
    int f0;  // kind 1: fold index of row block 0 (wrnn_set_fold_ranges): p = (f0 + f) * tpo + t
};
struct GemmB {  // B(k, n)
    int kind;   // 0: row-major [k*ld + n]; 1: im2col of the zero-padded mel (conv_in)
    const float* p;
    int ld;
    int T, pad, ksz;  // kind 1
};
struct GemmEp {
    int kind;   // 0: +bias[n]; 1: +bias[m]; 2: BN(m) [+relu] [+res];
                // 3: +bias[n] into folded row t * Btot + row0 + f (m = f * S + t, S = M / Bu)
    int Bu, Btot, row0;
    float* D;
    int ld;
    const float* bias;
    const float* alpha;
    const float* beta;
    const float* res;
    int relu;
};

// launch wrappers (kernels_*.hip); return hipError_t
hipError_t launch_stage(const StageArgs& a, int K, int RT, int NRG, int n_row_tiles,
                        hipStream_t s);
hipError_t prepare_stage(int K, int RT, int NRG);  // dynamic-LDS attribute (before capture)
hipError_t launch_sample(const SampleArgs& a, hipStream_t s);
hipError_t launch_noise_raw(float* q, int S, int nrows, int n_classes, const RowInfo* rows,
                            uint32_t k0, uint32_t k1, hipStream_t s);
hipError_t launch_gemm(int M, int N, int K, const GemmA& a, const GemmB& b, const GemmEp& e,
                       hipStream_t s);
hipError_t launch_mel_stencil(const float* in, int in_pad, int T_in, int W_in, float* out,
                              int scale, const float* w, int c, int out_lo, int out_len,
                              int ld_out, hipStream_t s);
hipError_t launch_fill_rows(float* dst, const float* src, int n, int rows, hipStream_t s);
// P1 [t][Btot][4 nq] of fold rows row0 .. row0 + Bu - 1 from the per-frame projections q / a
// ([1 + T][4 nq], slot 0 = zero frame) and the upsampler's per-phase taps [hop][8] (runtime.hip
// pack_p1): P1(p = hop f + s) = sum_k taps[s][k] q(f - 2 + k) + a(f), a(zero frame) for p >= L.
// Fold rows are f0 .. f0 + Bu - 1 of the utterance (positions (f0 + fo) * tpo + t).
hipError_t launch_p1_expand(float* P1, int Btot, int row0, int Bu, int f0, int S, int tpo, int L,
                            int hop, int T, int nq, const float* q, const float* a, const float* taps,
                            hipStream_t s);

// ---------------------------------------------------------------------------------------
// Persistent, weight-stationary fatchord recurrence (kernels_persist.hip). 8 XCD-local groups
// of 32 workgroups; in one launch group g owns fold rows rb+g, rb+g+8, ... rb+g+8(NR-1): the
// host pads the row count to a multiple of 8*NR and runs one launch per row batch when the
// rows exceed what one launch holds register-resident.
// ---------------------------------------------------------------------------------------
constexpr int kPG = 8;       // groups (one per XCD)
constexpr int kPM = 32;      // workgroups per group
constexpr int kPT = 512;     // threads per workgroup
constexpr int kPNR = 4;      // max fold rows per group -> B <= 32
constexpr int kPH = 512;     // rnn_dims == fc_dims
constexpr int kPK4 = kPH / 4;
constexpr int kPCls = 32;    // max classes per workgroup -> n_classes <= 1024
constexpr int kPPhases = 32; // diagnostic stamps per workgroup per traced step

// float4 weight registers per thread: 24 gate rows (stage A) + 8 fc1|fc2 rows [+ 8 fc3 rows
// when a workgroup owns more than 16 classes]; the rest of the slot's weights live in LDS.
inline int persist_reg_f4(int cpw) { return cpw > 16 ? 40 : 32; }
// LDS weights per slot (float4): W_hh2 [16 units][3][kPK4], then fc3 [16 classes][kPK4]
constexpr int kPLdsW4 = 16 * 3 * kPK4 + 16 * kPK4;
// Sparse instances (pruned weights): the slot's live 1 x 4 blocks as
// per-(set, output row) lists in the same kPLdsW4 float4; its last 16 float4 stay zero (the
// row a lane with no block left reads), so the lists hold at most kPSpZero float4
constexpr int kPSpZero = kPLdsW4 - 16;

// control words (zeroed by the host before every launch); PC_ERR: 1 registration timeout,
// 2 exchange timeout, 3 workgroups not spread 32 per XCD
// PC_WHERE: the first exchange timeout's site (wide kernel: site << 28 | slot << 22 | wave << 19),
// reported in the error message; PC_WHERE + 1: whether that poll's packets were missing;
// PC_WHERE + 2: its step
enum PersistCtl : int { PC_REG = 0, PC_TOTAL = 8, PC_ERR = 9, PC_WHERE = 10, PC_WORDS = 16 };
// progress cadence of the reference's callback (fatchord_version.py:234: i % 100 == 0)
constexpr int kProgressEvery = 100;
// host-mapped abort request word, kAbortWord words past the progress word (a cache line of its
// own): set by the host when the progress callback aborts (persist_common.h p_abort)
constexpr int kAbortWord = 16;
// PC_ERR codes: 1 registration timeout, 2 exchange timeout, 3 not spread 32 per XCD,
// 4 aborted by the host (progress callback)

struct PersistArgs {
    unsigned* ctl;          // PC_WORDS control words
    float* xbuf;            // per-group exchange area (persist_xbuf_floats())
    int t0, t1, S;          // steps [t0, t1) of S
    int B, nr, rb;          // B: row stride of every [t][row] array (padded rows);
                            // this launch runs rows rb + g + 8 r, r < nr (one row batch)
    int nreal;              // real rows: rows >= nreal are padding (their stream loads are
                            // redirected to row rb, so they cost no HBM traffic)
    int mode, n_classes, hop, cpw;  // cpw = classes per workgroup
    const RowInfo* rows;    // [B]
    const float4* wreg;     // [kPM][kPT][persist_reg_f4(cpw)]
    const float4* wlds;     // [kPM][kPLdsW4]
    const float* b_hh1;     // [3H]
    const float* b_hh2;     // [3H]
    const float* b_fc3;     // [n]
    const float* v;         // [3H] W_ih1 . w0
    const float* w0;        // [H]
    const float* fcond;     // per-frame conditioning rows
    int cond_width, oG2, oF1, oF2;
    const float* P1;        // [S][B][3H] = W_ih1 cI + b_ih1
    const float* cI;        // [S][B][H]
    // P1 ring (k_persist, when p1q != nullptr): P1 (r, z, n, cI) of step t + 2 is formed in the
    // launch by the unit's owner slot from the per-frame projections (runtime.hip pack_p1,
    // the same arithmetic as k_p1_expand) and handed to every slot through the exchange area;
    // then only k_persist_init reads P1 (step 0) and the [S][B][4H] stream is never written.
    const float* p1q;       // [frame slots][4H]: M1_mel mel(frame), slot fbase = zero frame
    const float* p1a;       // [frame slots][4H]: M1_aux aux(frame) + bP1 (zero frame: bP1)
    const float* p1taps;    // [hop][4]: upsampler taps of frames f-2+k0 .. f+1+k0 at phase s,
    int p1split;            // k0 = (s >= p1split)
    const float* gumbel;    // RAW [S][B][n] Gumbel noise; MOL [S][B][kMolNoise]
    int16_t* labels;        // [B][ld]
    float* samples;         // [B][ld]
    int ld;
    uint32_t k0, k1;        // Philox key (MOL draws in-kernel)
    float* st_x1;           // [B][H] chunk state: x1, h1 of step t0 ...
    float* st_h1;
    float* st_h2;           // ... h2 and gh2 = W_hh2 h2 + b_hh2 after step t0-1
    float* st_gh2;          // [B][3H]
    uint32_t* stamps;       // optional: [0] loop start, [1] loop end (group 0, slot 0)
    uint32_t* phases;       // optional: [256][kPPhases] stamps of step phase_t
    int phase_t;
    unsigned* progress;     // optional host-mapped word: steps done (persist_common.h p_progress)
    int prog_base;          // row batch * S
    // wide-row launches (kernels_persist_wide.hip): MFMA A-operand weight images
    const float4* wwide;    // [kPM][8 waves][40 float4][64 lanes]
    const float4* wwide_lds;// [kPM][2 tiles][8][4][64] (W_hh2 z, n)
    const float4* wfc3b;    // > 512 classes: fc3 rows 512 + 16 w + i, [kPM][8 waves][4][64 lanes]
    float* wring;           // runtimeracer wide launches: per-group ring of P1 and noise
    DbgLogits dbg;
    // rotated launch (k_persist; null otherwise): virtual row v = g + 8 r ->
    // (physical row, step offset), rows per group (nr or nr - 1), steps per group; `rows` is then
    // the launch's RowInfo table by virtual row (rel0 advanced by the offset)
    const int2* vmap;
    const int* gnr;
    const int* giters;
    // sparse instance (k_persist only; P1 ring): wreg = [kPM][kPT] uint4 per-lane masks / list
    // bases, wlds = [kPM][kPLdsW4] float4 block lists (runtime.hip pack_persist_sparse)
    int sparse;
};

hipError_t launch_persist(const PersistArgs& a, hipStream_t s);
// Wide-row fatchord launch: up to kPWideRows rows per XCD group (8 kPWideRows per launch),
// fp32 MFMA products, RAW categorical with <= 1024 classes (> 512: PersistArgs::wfc3b).
constexpr int kPWideRows = 16;
hipError_t launch_persist_wide(const PersistArgs& a, hipStream_t s);
size_t persist_wide_lds_bytes();
size_t persist_wide_xbuf_floats();
hipError_t persist_wide_reset_xbuf(float* xbuf, hipStream_t s);
size_t persist_wide_ring_floats();
size_t persist_wide_wreg_floats();
size_t persist_wide_wlds_floats();
int persist_wide_scratch(bool c10 = false);      // (c10: the 1024-class instances)
int persist_wide_rot_scratch(bool c10 = false);  // the time-sliced instance (PersistArgs::vmap)
int wide_layout_check(int rows_per_group);  // host: violations of the exchange layout (wide_layout.h)
hipError_t launch_persist_init(const PersistArgs& a, hipStream_t s);
constexpr int kMolNoise = 12;  // floats per (step, row) of the precomputed MOL noise
// ---------------------------------------------------------------------------------------
// Persistent runtimeracer recurrence (kernels_persist_rr.hip): rnn_dims = fc_dims = 256, four
// GRUs and five linears per step. Same 8 XCD-local groups x 32 workgroups x 512 threads; a
// workgroup owns 8 units / outputs of every layer and cpw classes of fc5; eight in-group hops
// per step (GRU2, GRU3, GRU4, fc1, fc2, fc3, fc4, fc5 candidates).
// ---------------------------------------------------------------------------------------
constexpr int kRH = 256;     // rnn_dims == fc_dims
constexpr int kRNR = 4;      // max fold rows per group and launch
constexpr int kRNW = 28;     // float4 weight registers per thread
constexpr int kRRState = 14; // chunk-state floats per row / H: x1, h1, h2, h3, h4 | gh2, gh3, gh4

struct PersistRRArgs {
    unsigned* ctl;          // PC_WORDS control words
    float* xbuf;            // per-group exchange area (persist_rr_xbuf_floats())
    int t0, t1, S;
    int B, nr, rb;          // row stride, rows per group, first row of this launch's batch
    int mode, n_classes, hop, cpw;
    const RowInfo* rows;
    const float4* wreg;     // [kPM][kPT][kRNW]
    const float4* w5;       // [kPM][32][kRH / 4] fc5 rows of each slot (LDS-resident)
    const float* b_ih2;     // [3H]
    const float* b_ih4;     // [3H]
    const float* b_hh1;     // [3H] ... b_hh4
    const float* b_hh2;
    const float* b_hh3;
    const float* b_hh4;
    const float* b_f2;      // [F]
    const float* b_f4;      // [F]
    const float* b_f5;      // [n]
    const float* v;         // [3H] W_ih1 . w0
    const float* w0;        // [H]
    const float* fcond;     // per-frame conditioning rows
    int cond_width, oG3, oF1, oF3;
    const float* P1;        // [S][B][3H]
    const float* cI;        // [S][B][H]
    const float* gumbel;    // RAW [S][B][n]; MOL [S][B][kMolNoise]
    int16_t* labels;        // [B][ld]
    float* samples;         // [B][ld]
    int ld;
    float* st;              // chunk state [B][kRRState H]: x1, h1, h2, h3, h4 | gh2, gh3, gh4 (3H each;
                            // gh4: the wide kernel's time-sliced launches only)
    uint32_t* stamps;       // optional: [0] loop start, [1] loop end (group 0, slot 0)
    unsigned* progress;     // as PersistArgs
    int prog_base;
    DbgLogits dbg;
    // wide-row launches (kernels_persist_wide_rr.hip): MFMA A-operand images, the per-slot ring
    // of P1 and noise, P1's per-frame form (as PersistArgs; p1q null: the P1 stream), Philox key
    const float4* wwide;    // [kPM][8 waves][30 float4][64 lanes]
    float* wring;           // persist_wide_rr_ring_floats()
    const float* p1q;
    const float* p1a;
    const float* p1taps;
    int p1split;
    uint32_t k0, k1;
    uint32_t* phases;       // optional: [256][kPPhases] stamps of step phase_t (wide: slots 0, 16)
    int phase_t;
    // time-sliced wide launch or rotated register-resident launch (§3.0e; null
    // otherwise): virtual row v = g + 8 r -> (physical row, step offset); `rows` is then the
    // launch's RowInfo table by virtual row; rotated: rows and steps per group
    const int2* vmap;
    const int* gnr;
    const int* giters;
};

hipError_t launch_persist_rr(const PersistRRArgs& a, hipStream_t s);
int persist_rr_rot_scratch(int nr, bool mol);  // the rotated RAW / MOL instance's scratch bytes (-1: none)
// Wide-row runtimeracer launch (kernels_persist_wide_rr.hip): up to kPWideRows rows per XCD
// group, the group split into two halves of 16 slots that own 16 units of alternate layers,
// fp32 MFMA products, RAW categorical with 512 or 1024 classes (cpw = n / 16 per B slot).
hipError_t launch_persist_wide_rr(const PersistRRArgs& a, hipStream_t s);
size_t persist_wide_rr_lds_bytes();
size_t persist_wide_rr_xbuf_floats();
size_t persist_wide_rr_ring_floats();
size_t persist_wide_rr_wreg_floats();
hipError_t persist_wide_rr_reset_xbuf(float* xbuf, hipStream_t s);
int persist_wide_rr_scratch();
int persist_wide_rr_rot_scratch();  // the time-sliced instance (PersistRRArgs::vmap)
int wide_rr_layout_check(int rows_per_group);

// ---------------------------------------------------------------------------------------
// Persistent geneing recurrence (kernels_persist_gen.hip): rnn_dims 256, fc_dims 128; per
// step fc1 (hop 1) and fc3 candidates (hop 2), W_hh1 h1 published as tagged pairs beside.
// ---------------------------------------------------------------------------------------
constexpr int kGF = 128;     // fc_dims
constexpr int kGNW = 16;     // float4 weight registers per thread

struct PersistGenArgs {
    unsigned* ctl;
    float* xbuf;            // per-group exchange area (persist_gen_xbuf_floats())
    int t0, t1, S;
    int B, nr, rb;
    int mode, n_classes, hop, cpw;
    const RowInfo* rows;
    const float4* wreg;     // [kPM][kPT][kGNW]
    const float* b_hh1;     // [3H]
    const float* b_f3;      // [n]
    const float* v;         // [3H] W_ih1 . w0
    const float* w0;        // [H]
    const float* fcond;     // per-frame conditioning rows (fc1: W_fc1[:, H:] a2 + b_fc1)
    int cond_width, oF1;
    const float* P1;        // [S][B][3H]
    const float* cI;        // [S][B][H]
    const float* gumbel;    // RAW [S][B][n]; MOL [S][B][kMolNoise]
    int16_t* labels;        // [B][ld]
    float* samples;         // [B][ld]
    int ld;
    float* st;              // chunk state [B][2 H]: x1, h1
    uint32_t* stamps;
    unsigned* progress;     // as PersistArgs
    uint32_t k0, k1;        // Philox key (BETA draws in-kernel)
    int prog_base;
    DbgLogits dbg;
    // rotated launch (BITS / MOL; null otherwise): virtual row v = g + 8 r ->
    // (physical row, step offset), `rows` the launch's RowInfo table by virtual row, rows and
    // steps per group
    const int2* vmap;
    const int* gnr;
    const int* giters;
};

hipError_t launch_persist_gen(const PersistGenArgs& a, hipStream_t s);
int persist_gen_rot_scratch(int nr, int mode);  // the rotated BITS / MOL instance's scratch bytes (-1: none)
hipError_t launch_persist_gen_init(const PersistGenArgs& a, hipStream_t s);
int persist_gen_variant_ok(int nr, int cpw, int mode);
size_t persist_gen_lds_bytes();
size_t persist_gen_xbuf_floats();
hipError_t launch_persist_rr_init(const PersistRRArgs& a, hipStream_t s);
int persist_rr_variant_ok(int nr, int cpw, int mode);
size_t persist_rr_lds_bytes();
size_t persist_rr_xbuf_floats();

hipError_t launch_mol_noise(float* out, int S, int nrows, const RowInfo* rows, uint32_t k0,
                            uint32_t k1, hipStream_t s);
hipError_t launch_gumbel(float* g, int S, int nrows, int n_classes, const RowInfo* rows,
                         uint32_t k0, uint32_t k1, hipStream_t s);
hipError_t launch_gumbel_rows(float* g, int S, int r0, int nrows, int ld, int n_classes,
                              const RowInfo* rows, uint32_t k0, uint32_t k1, hipStream_t s);
// ring: the P1-ring variant (PersistArgs::p1q set) or the P1-stream variant
int persist_variant_ok(int nr, int cpw, int mode, int ring);
int persist_variant_scratch(int nr, int cpw, int mode, int ring, int sparse = 0);
// rotated instance (groups of nr and nr - 1 rows)
int persist_rot_scratch(int nr, int mode, int sparse = 0);
size_t persist_lds_bytes();
size_t persist_xbuf_floats();

}  // namespace wrnn
