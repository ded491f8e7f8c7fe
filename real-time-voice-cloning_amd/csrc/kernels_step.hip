// Recurrent-step kernels of the MI355X WaveRNN vocoder.
//
// One autoregressive step of WaveRNN.generate (reference: vocoder/models/fatchord_version.py
// :192-236, runtimeracer_version.py:242-291) is a chain of "stage" launches. Each stage is one
// all-to-all seam of the recurrence: it computes a fp32 matrix-vector product for every fold
// row (the batch) plus the elementwise layer that follows it (GRU gates, bias, ReLU), and may
// carry extra independent segments (W_hh h for the next step, W_ih1 cI for the next step) that
// are off the critical path. The chain is captured in HIP graphs by runtime.hip.
//
// Tile scheme (256 threads): a workgroup owns OT outputs of one segment for RT fold rows.
// Its weight tile is loaded once into registers (packed so each wave reads contiguous
// memory), the RT x K input rows are staged in LDS, every thread accumulates OPL x RT
// partial dot products over its k-chunk (fma chain in ascending k), the partials are reduced
// across k-chunks through LDS in a fixed order (deterministic), and the epilogue is applied by
// the thread that owns the final (unit, row) pair.
#include "wrnn_kernels.h"
#include "philox.h"
#include "cand_key.h"

namespace wrnn {

__device__ __forceinline__ void phase_stamp(uint32_t* ph, int i) {
    if (ph && threadIdx.x == 0) {
        const int wg = blockIdx.y * gridDim.x + blockIdx.x;
        if (wg < kMaxStampWG) ph[8 * wg + i] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
}

__device__ __forceinline__ int frame_of(const RowInfo& ri, int t, int hop) {
    const int rel = ri.rel0 + t;
    return rel < ri.L ? ri.fbase + 1 + rel / hop : ri.fbase;
}

__device__ __forceinline__ float sigmoid_ref(float x) {
    // torch CPU sigmoid: 1 / (1 + exp(-x))
    return 1.0f / (1.0f + expf(-x));
}

// torch GRUCell (aten/native/RNN.cpp GRUCell): r = sig(gh_r + gi_r), z = sig(gh_z + gi_z),
// n = tanh(gi_n + gh_n * r), h' = (h - n) * z + n  -- separate roundings, no contraction.
__device__ __forceinline__ float gru_cell(float gi_r, float gi_z, float gi_n, float gh_r,
                                          float gh_z, float gh_n, float h) {
#pragma clang fp contract(off)
    const float r = sigmoid_ref(gh_r + gi_r);
    const float z = sigmoid_ref(gh_z + gi_z);
    const float ghr = gh_n * r;
    const float n = tanhf(gi_n + ghr);
    const float d = h - n;
    const float dz = d * z;
    return dz + n;
}

__device__ __forceinline__ float add_nc(float a, float b) {
#pragma clang fp contract(off)
    return a + b;
}

template <int K, int RT, int NRG, int CFG>
__device__ __forceinline__ void seg_tile(const StageArgs& a, const Seg& sg, int tile, int row0,
                                         float* lds) {
    constexpr int OPL = CFG == TILE_GATE ? 3 : 1;
    constexpr int NOG = kTileNOG;
    constexpr int KC = kThreads / (NOG * NRG);  // k-chunks
    constexpr int KR = K / KC;                  // k per thread
    constexpr int BR = RT / NRG;                // rows per thread
    constexpr int KCP = KC + 4;  // padded reduction row: conflict-free ds_read_b128 per row
    constexpr int NX = (RT * (K / 4) + kThreads - 1) / kThreads;  // X float4 per thread
    static_assert(KR % 4 == 0 && KC % 4 == 0 && RT % NRG == 0, "bad tile shape");
    static_assert(NOG * RT <= kThreads, "one epilogue pair per thread");
    const int tid = threadIdx.x;
    const int og = tid % NOG, rg = (tid / NOG) % NRG, kc = tid / (NOG * NRG);
    const int nrows = a.nrows;
    const int H = sg.H;
    const bool gather = sg.x_pld != 0;

    // ---- 1. issue every global load of this tile up front (latency overlaps) ------------
    // weight tile -> registers; packed [tile][kc][og][j][kk] (row groups share a slice)
    float4 wv[OPL * KR / 4];
    {
        const float4* wp = reinterpret_cast<const float4*>(
            sg.W + (((size_t)tile * KC + kc) * NOG + og) * (size_t)(OPL * KR));
#pragma unroll
        for (int i = 0; i < OPL * KR / 4; ++i) wv[i] = wp[i];
    }
    // input rows -> registers (staged to LDS below)
    float4 xv[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        const int e = tid + i * kThreads;
        const int b = e / (K / 4), q = e % (K / 4);
        const int r = row0 + b;
        xv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < RT * (K / 4) && r < nrows) {
            long long off = sg.x_off + (long long)r * sg.x_ld;
            if (gather) off += (long long)a.rows[r].pos0 * sg.x_pld;
            xv[i] = reinterpret_cast<const float4*>(sg.X + off)[q];
        }
    }
    // epilogue operands of this thread's (group, row) pair
    const int pog = tid / RT, pb = tid % RT;
    const int pr = row0 + pb;
    const bool has_pair = tid < NOG * RT && pr < nrows;
    float e_c[OPL], e_gh[3] = {0.f, 0.f, 0.f}, e_h = 0.f, e_x = 0.f;
#pragma unroll
    for (int j = 0; j < OPL; ++j) e_c[j] = 0.f;
    const int e_o = tile * NOG + pog;  // unit (TILE_GATE) or output (TILE_OUT)
    if (has_pair) {
        const float* cr = sg.cond;
        if (sg.c_ld) cr += (size_t)frame_of(a.rows[pr], a.t, a.hop) * (size_t)sg.c_ld;
        if constexpr (CFG == TILE_GATE) {
            if (e_o < H) {
#pragma unroll
                for (int j = 0; j < 3; ++j) e_c[j] = cr[j * H + e_o];
                if (sg.kind == EPI_GRU) {
                    const float* gh = sg.gh + (size_t)pr * 3 * H;
#pragma unroll
                    for (int j = 0; j < 3; ++j) e_gh[j] = gh[j * H + e_o];
                    e_h = sg.h[(size_t)pr * H + e_o];
                    long long off = sg.x_off + (long long)pr * sg.x_ld;
                    if (gather) off += (long long)a.rows[pr].pos0 * sg.x_pld;
                    e_x = sg.X[off + e_o];
                }
            }
        } else {
            if (e_o < sg.n_out) e_c[0] = cr[e_o];
        }
    }

    // ---- 2. stage X in LDS: Xs[b][K] ---------------------------------------------------
    float4* Xs4 = reinterpret_cast<float4*>(lds);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
        const int e = tid + i * kThreads;
        if (e < RT * (K / 4)) Xs4[e] = xv[i];
    }
    __syncthreads();
    phase_stamp(a.phases, 1);

    // ---- 3. partial dot products over this thread's k-chunk (fma chain, ascending k) ----
    float acc[OPL][BR];
#pragma unroll
    for (int j = 0; j < OPL; ++j)
#pragma unroll
        for (int i = 0; i < BR; ++i) acc[j][i] = 0.f;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
        const int b = rg * BR + i;
#pragma unroll
        for (int q = 0; q < KR / 4; ++q) {
            const float4 x4 = Xs4[b * (K / 4) + kc * (KR / 4) + q];
#pragma unroll
            for (int j = 0; j < OPL; ++j) {
                const float4 w4 = wv[j * (KR / 4) + q];
                float s = acc[j][i];
                s = fmaf(w4.x, x4.x, s);
                s = fmaf(w4.y, x4.y, s);
                s = fmaf(w4.z, x4.z, s);
                s = fmaf(w4.w, x4.w, s);
                acc[j][i] = s;
            }
        }
    }
    phase_stamp(a.phases, 2);
    __syncthreads();

    // ---- 4. partials -> LDS red[og][j][b][kc] (kc contiguous, rows padded) --------------
    float* red = lds;
#pragma unroll
    for (int j = 0; j < OPL; ++j)
#pragma unroll
        for (int i = 0; i < BR; ++i)
            red[((og * OPL + j) * RT + rg * BR + i) * KCP + kc] = acc[j][i];
    __syncthreads();
    phase_stamp(a.phases, 3);

    // ---- 5. reduce over k-chunks in kc order and apply the epilogue ---------------------
    if (!has_pair) return;
    float s[OPL];
#pragma unroll
    for (int j = 0; j < OPL; ++j) {
        const float4* rp = reinterpret_cast<const float4*>(red + ((pog * OPL + j) * RT + pb) * KCP);
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < KC / 4; ++c) {
            const float4 t4 = rp[c];
            v += t4.x;
            v += t4.y;
            v += t4.z;
            v += t4.w;
        }
        s[j] = v;
    }
    if constexpr (CFG == TILE_GATE) {
        if (e_o >= H) return;
        if (sg.kind == EPI_GRU) {
            const float gi_r = add_nc(s[0], e_c[0]);
            const float gi_z = add_nc(s[1], e_c[1]);
            const float gi_n = add_nc(s[2], e_c[2]);
            const float hn = gru_cell(gi_r, gi_z, gi_n, e_gh[0], e_gh[1], e_gh[2], e_h);
            sg.h[(size_t)pr * H + e_o] = hn;
            sg.xout[(size_t)pr * H + e_o] = add_nc(e_x, hn);
        } else {  // EPI_BIAS3
            float* y = sg.Y + (size_t)pr * sg.y_ld;
#pragma unroll
            for (int j = 0; j < 3; ++j) y[j * H + e_o] = add_nc(s[j], e_c[j]);
        }
    } else {
        if (e_o < sg.n_out) {
            float v = add_nc(s[0], e_c[0]);
            if (sg.kind == EPI_COND_RELU) v = v > 0.f ? v : 0.f;
            sg.Y[(size_t)pr * sg.y_ld + e_o] = v;
        }
    }
}

template <int K, int RT, int NRG>
__global__ __launch_bounds__(kThreads) void k_stage(StageArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    uint32_t t_begin = 0;
    if (a.stamps) t_begin = (uint32_t)__builtin_amdgcn_s_memrealtime();
    phase_stamp(a.phases, 0);
    const int bx = blockIdx.x;
    const int row0 = blockIdx.y * RT;
    int s = 0;
    while (s + 1 < a.nseg && bx >= a.tile_start[s + 1]) ++s;
    const Seg& sg = a.seg[s];
    const int tile = bx - a.tile_start[s];
    if (sg.cfg == TILE_GATE)
        seg_tile<K, RT, NRG, TILE_GATE>(a, sg, tile, row0, lds);
    else
        seg_tile<K, RT, NRG, TILE_OUT>(a, sg, tile, row0, lds);
    if (a.phases) {
        __syncthreads();
        phase_stamp(a.phases, 4);
    }
    if (a.stamps) {
        __syncthreads();
        const int wg = blockIdx.y * gridDim.x + blockIdx.x;
        if (threadIdx.x == 0 && wg < kMaxStampWG) {
            a.stamps[2 * wg] = t_begin;
            a.stamps[2 * wg + 1] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        }
    }
}

template <int K, int RT, int NRG>
static size_t stage_lds_bytes() {
    const size_t xs = (size_t)RT * K * sizeof(float);
    const size_t kcp = kThreads / (kTileNOG * NRG) + 4;
    const size_t red = (size_t)kTileNOG * 3 * RT * kcp * sizeof(float);
    return xs > red ? xs : red;
}

template <int K, int RT, int NRG>
static hipError_t prepare_stage_t() {
    return hipFuncSetAttribute((const void*)k_stage<K, RT, NRG>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)stage_lds_bytes<K, RT, NRG>());
}

template <int K, int RT, int NRG>
static hipError_t launch_stage_t(const StageArgs& a, int n_row_tiles, hipStream_t s) {
    const int n_tiles = a.tile_start[a.nseg];
    const size_t lds = stage_lds_bytes<K, RT, NRG>();
    hipLaunchKernelGGL((k_stage<K, RT, NRG>), dim3(n_tiles, n_row_tiles), dim3(kThreads), lds, s,
                       a);
    return hipGetLastError();
}

template <int K, int RT>
static hipError_t dispatch_nrg(bool prep, const StageArgs* a, int NRG, int nrt, hipStream_t s) {
    switch (NRG) {  // K = 128 needs NRG >= 2 (4 k per thread; the runtime packs for that)
        case 1:
            if constexpr (K >= 256)
                return prep ? prepare_stage_t<K, RT, 1>() : launch_stage_t<K, RT, 1>(*a, nrt, s);
            return hipErrorInvalidValue;
        case 2: return prep ? prepare_stage_t<K, RT, 2>() : launch_stage_t<K, RT, 2>(*a, nrt, s);
        case 4: return prep ? prepare_stage_t<K, RT, 4>() : launch_stage_t<K, RT, 4>(*a, nrt, s);
        default: return hipErrorInvalidValue;
    }
}

template <int K>
static hipError_t dispatch_rt(bool prep, const StageArgs* a, int RT, int NRG, int nrt,
                              hipStream_t s) {
    switch (RT) {
        case 4: return dispatch_nrg<K, 4>(prep, a, NRG, nrt, s);
        case 8: return dispatch_nrg<K, 8>(prep, a, NRG, nrt, s);
        case 12: return dispatch_nrg<K, 12>(prep, a, NRG, nrt, s);
        case 16: return dispatch_nrg<K, 16>(prep, a, NRG, nrt, s);
        case 20: return dispatch_nrg<K, 20>(prep, a, NRG, nrt, s);
        case 24: return dispatch_nrg<K, 24>(prep, a, NRG, nrt, s);
        case 32: return dispatch_nrg<K, 32>(prep, a, NRG, nrt, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t prepare_stage(int K, int RT, int NRG) {
    if (K == 512) return dispatch_rt<512>(true, nullptr, RT, NRG, 0, nullptr);
    if (K == 256) return dispatch_rt<256>(true, nullptr, RT, NRG, 0, nullptr);
    if (K == 128) return dispatch_rt<128>(true, nullptr, RT, NRG, 0, nullptr);
    return hipErrorInvalidValue;
}

hipError_t launch_stage(const StageArgs& a, int K, int RT, int NRG, int n_row_tiles,
                        hipStream_t s) {
    if (K == 512) return dispatch_rt<512>(false, &a, RT, NRG, n_row_tiles, s);
    if (K == 256) return dispatch_rt<256>(false, &a, RT, NRG, n_row_tiles, s);
    if (K == 128) return dispatch_rt<128>(false, &a, RT, NRG, n_row_tiles, s);
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------
// Sampling + GRU1 of the next step (one workgroup per fold row).
// Wave reductions use DPP (quad_perm / row_ror inside 16-lane rows, readlane across rows);
// the order of every reduction is fixed, so results are run-to-run deterministic.
// ---------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ float lanef(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppRor4 = 0x124, kDppRor8 = 0x128;

__device__ __forceinline__ float wave_max_all(float v) {
    v = fmaxf(v, dppf<kDppXor1>(v));
    v = fmaxf(v, dppf<kDppXor2>(v));
    v = fmaxf(v, dppf<kDppRor4>(v));
    v = fmaxf(v, dppf<kDppRor8>(v));
    return fmaxf(fmaxf(lanef(v, 0), lanef(v, 16)), fmaxf(lanef(v, 32), lanef(v, 48)));
}
__device__ __forceinline__ float wave_sum_all(float v) {
    v += dppf<kDppXor1>(v);
    v += dppf<kDppXor2>(v);
    v += dppf<kDppRor4>(v);
    v += dppf<kDppRor8>(v);
    return ((lanef(v, 0) + lanef(v, 16)) + lanef(v, 32)) + lanef(v, 48);
}
__device__ __forceinline__ void amax_step(float& v, int& i, float v2, int i2) {
    const bool take = (v2 > v) | ((v2 == v) & (i2 < i));  // bitwise: no exec-mask branches
    v = take ? v2 : v;
    i = take ? i2 : i;
}
template <int CTRL>
__device__ __forceinline__ void amax_dpp(float& v, int& i) {
    amax_step(v, i, dppf<CTRL>(v), dppi<CTRL>(i));
}
__device__ __forceinline__ void wave_argmax_all(float& v, int& i) {
    amax_dpp<kDppXor1>(v, i);
    amax_dpp<kDppXor2>(v, i);
    amax_dpp<kDppRor4>(v, i);
    amax_dpp<kDppRor8>(v, i);
    float bv = lanef(v, 0);
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int l = 16; l < 64; l += 16)
        amax_step(bv, bi, lanef(v, l), __builtin_amdgcn_readlane(i, l));
    v = bv;
    i = bi;
}

constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ float block_max(float v, float* sh) {
    v = wave_max_all(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = sh[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) r = fmaxf(r, sh[w]);
    __syncthreads();
    return r;
}
__device__ __forceinline__ float block_sum(float v, float* sh) {
    v = wave_sum_all(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = sh[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) r += sh[w];
    __syncthreads();
    return r;
}

constexpr int kMaxClassesPerThread = 16;  // n_classes <= 4096 (bits <= 12)
constexpr int kMaxUnits = 4;              // H <= 1024

__global__ __launch_bounds__(kThreads) void k_sample(SampleArgs a) {
    __shared__ int shi[2 * kWaves];
    __shared__ float xsh;
    __shared__ uint32_t words[12];
    const int r = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    phase_stamp(a.phases, 0);
    const int H = a.H;
    const int n = a.n_classes;
    const RowInfo ri = a.rows[r];
    // 1. loads that do not depend on the sample: logits, GRU1 operands of step t+1
    float l[kMaxClassesPerThread];
    if (a.t >= 0 && a.mode == 0) {
        const float* lg = a.logits + (size_t)r * n;
#pragma unroll
        for (int i = 0; i < kMaxClassesPerThread; ++i) {
            const int k = tid + i * kThreads;
            l[i] = k < n ? lg[k] : -INFINITY;
        }
    }
    float g_P[kMaxUnits][3], g_gh[kMaxUnits][3], g_v[kMaxUnits][3], g_h[kMaxUnits],
        g_c[kMaxUnits], g_w[kMaxUnits];
    if (a.do_gru) {
        // folded conditioning: cI rows of step t+1 are contiguous ([t][row][H])
        const float* P1 = a.P1 + (size_t)r * 3 * H;
        const float* gh = a.gh1 + (size_t)r * 3 * H;
        const float* cI = a.cI + ((size_t)(a.t + 1) * a.nrows + r) * H;
#pragma unroll
        for (int i = 0; i < kMaxUnits; ++i) {
            const int j = tid + i * kThreads;
            if (j < H) {
#pragma unroll
                for (int g = 0; g < 3; ++g) {
                    g_P[i][g] = P1[g * H + j];
                    g_gh[i][g] = gh[g * H + j];
                    g_v[i][g] = a.v[g * H + j];
                }
                g_h[i] = a.h1[(size_t)r * H + j];
                g_c[i] = cI[j];
                g_w[i] = a.w0[j];
            }
        }
    }
    // teacher-forced logit gate (debug only): this row's logits at a recorded step
    if (a.t >= 0 && a.dbg.out != nullptr) {
        const int k = a.dbg.map[a.t];
        if (k >= 0)
            for (int c = tid; c < n; c += kThreads)
                a.dbg.out[((size_t)k * a.nrows + r) * n + c] = a.logits[(size_t)r * n + c];
    }
    float x = 0.f;
    if (a.t >= 0) {
        if (a.mode == 0) {
            // 2. the decision (cand_key.h cand_key, the same as the persistent kernels'):
            //    argmax_k (l_k + G_k), G_k = -log q_k of the contract's Exp(1) variate (philox.h
            //    gumbel_q_of, computed while the logits are in flight), l + G formed exactly --
            //    the reference's argmax((softmax(l) / sum) / q) without fp32 rounding of its own
            uint32_t gq[kMaxClassesPerThread];
#pragma unroll
            for (int i = 0; i < kMaxClassesPerThread; ++i) {
                const int k = tid + i * kThreads;
                gq[i] = 0u;
                if (k < n) {
                    const U4 o = philox4x32_10((uint32_t)(k >> 2), (uint32_t)a.t, (uint32_t)ri.fold, ri.stream,
                                               a.k0, a.k1);
                    const uint32_t w = (k & 3) == 0 ? o.x : (k & 3) == 1 ? o.y : (k & 3) == 2 ? o.z : o.w;
                    gq[i] = gumbel_q_of(w);
                }
            }
            uint32_t bh = 0u, bl = 0u;
#pragma unroll
            for (int i = 0; i < kMaxClassesPerThread; ++i) {
                const int k = tid + i * kThreads;
                if (k < n) {
                    const CandKey c = cand_key(l[i], gq[i], k);
                    kmax_take(bh, bl, c.hi, c.lo);
                }
            }
            // wave: DPP rows, then the 4 row results; workgroup: the waves' results via LDS
            row16_kmax(bh, bl);
#pragma unroll
            for (int rr = 16; rr < 64; rr += 16)
                kmax_take(bh, bl, (uint32_t)__builtin_amdgcn_readlane((int)bh, rr), (uint32_t)__builtin_amdgcn_readlane((int)bl, rr));
            if (lane == 0) {
                shi[wv] = (int)bh;
                shi[kWaves + wv] = (int)bl;
            }
            __syncthreads();
            bh = (uint32_t)shi[0];
            bl = (uint32_t)shi[kWaves];
#pragma unroll
            for (int w = 1; w < kWaves; ++w) kmax_take(bh, bl, (uint32_t)shi[w], (uint32_t)shi[kWaves + w]);
            const int bk = key_cls(bl);
            {
#pragma clang fp contract(off)
                x = (2.0f * (float)bk) / (float)(n - 1) - 1.0f;
            }
            if (tid == 0) {
                a.labels[(size_t)r * a.S + a.t] = (int16_t)bk;
                a.samples[(size_t)r * a.S + a.t] = x;
            }
        } else if (a.mode == 2) {
            // BETA (geneing 'RAW'): vocoder/distribution.py:7-20, Beta(exp l0, exp l1) on [-1, 1]
            // lanes 0 / 1 draw the two gammas concurrently (philox.h gamma_mt); lane 0 forms
            // 2 X / (X + Y) - 1 exactly as beta_sample does
            if (tid < 64) {
                double gv = 0.0;
                if (lane < 2)
                    gv = gamma_mt((double)expf(a.logits[(size_t)r * n + lane]), (uint32_t)lane,
                                  (uint32_t)a.t, (uint32_t)ri.fold, ri.stream, a.k0, a.k1);
                const double gy = __shfl(gv, 1);
                if (lane == 0) {
#pragma clang fp contract(off)
                    const float sb = (float)(gv / (gv + gy));
                    const float xv = 2.0f * sb - 1.0f;
                    a.samples[(size_t)r * a.S + a.t] = xv;
                    xsh = xv;
                }
            }
            __syncthreads();
            x = xsh;
        } else {
            // MOL: vocoder/distribution.py:104-140 with the Philox draws
            const float* lg = a.logits + (size_t)r * n;
            if (tid < 3) {
                const U4 o = philox4x32_10(kMolDomain | (uint32_t)tid, (uint32_t)a.t,
                                           (uint32_t)ri.fold, ri.stream, a.k0, a.k1);
                words[4 * tid + 0] = o.x;
                words[4 * tid + 1] = o.y;
                words[4 * tid + 2] = o.z;
                words[4 * tid + 3] = o.w;
            }
            __syncthreads();
            if (wv == 0) {
                float v = -INFINITY;
                int idx = 0x7fffffff;
                if (lane < 10) {
#pragma clang fp contract(off)
                    const float u1 = mol_uniform_from_u32(words[lane]);
                    v = lg[lane] - logf(-logf(u1));
                    idx = lane;
                }
                wave_argmax_all(v, idx);
                if (lane == 0) {
#pragma clang fp contract(off)
                    const float u2 = mol_uniform_from_u32(words[10]);
                    const float mean = lg[10 + idx];
                    float ls = lg[20 + idx];
                    const float lsmin = -32.23619130191664f;  // float(np.log(1e-14))
                    ls = ls < lsmin ? lsmin : ls;
                    const float lu = logf(u2) - logf(1.0f - u2);
                    float xv = mean + expf(ls) * lu;
                    xv = xv < -1.f ? -1.f : xv;
                    xv = xv > 1.f ? 1.f : xv;
                    a.samples[(size_t)r * a.S + a.t] = xv;
                    xsh = xv;
                }
            }
            __syncthreads();
            x = xsh;
        }
    }
    phase_stamp(a.phases, 1);
    if (!a.do_gru) return;
    // 4. GRU1 of step t+1: gi = W_ih1 (cI + w0 x) + b_ih1 = P1 + v x ; xI = cI + w0 x
#pragma unroll
    for (int i = 0; i < kMaxUnits; ++i) {
        const int j = tid + i * kThreads;
        if (j < H) {
            const float gi_r = fmaf(g_v[i][0], x, g_P[i][0]);
            const float gi_z = fmaf(g_v[i][1], x, g_P[i][1]);
            const float gi_n = fmaf(g_v[i][2], x, g_P[i][2]);
            const float hn = gru_cell(gi_r, gi_z, gi_n, g_gh[i][0], g_gh[i][1], g_gh[i][2], g_h[i]);
            const float xI = fmaf(g_w[i], x, g_c[i]);
            a.h1[(size_t)r * H + j] = hn;
            a.x1[(size_t)r * H + j] = add_nc(xI, hn);
        }
    }
    if (a.phases) {
        __syncthreads();
        phase_stamp(a.phases, 2);
    }
}

hipError_t launch_sample(const SampleArgs& a, hipStream_t s) {
    if (a.mode == 0 && a.n_classes > kMaxClassesPerThread * kThreads) return hipErrorInvalidValue;
    if (a.H > kMaxUnits * kThreads) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_sample, dim3(a.nrows), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// RAW noise: q[t][r][k] = Exp(1) from Philox(k>>2, t, fold, stream; seed)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_noise_raw(float4* q, int S, int nrows, int ng,
                                                        const RowInfo* rows, uint32_t k0,
                                                        uint32_t k1) {
    const long long gid = (long long)blockIdx.x * kThreads + threadIdx.x;
    const long long total = (long long)S * nrows * ng;
    if (gid >= total) return;
    const int g = (int)(gid % ng);
    const long long tr = gid / ng;
    const int r = (int)(tr % nrows);
    const int t = (int)(tr / nrows);
    const U4 o = philox4x32_10((uint32_t)g, (uint32_t)t, (uint32_t)rows[r].fold, rows[r].stream,
                               k0, k1);
    q[gid] = make_float4(exp1_from_u32(o.x), exp1_from_u32(o.y), exp1_from_u32(o.z),
                         exp1_from_u32(o.w));
}

hipError_t launch_noise_raw(float* q, int S, int nrows, int n_classes, const RowInfo* rows,
                            uint32_t k0, uint32_t k1, hipStream_t s) {
    if (n_classes % 4) return hipErrorInvalidValue;
    const int ng = n_classes / 4;
    const long long total = (long long)S * nrows * ng;
    const long long blocks = (total + kThreads - 1) / kThreads;
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_noise_raw, dim3((unsigned)blocks), dim3(kThreads), 0, s,
                       reinterpret_cast<float4*>(q), S, nrows, ng, rows, k0, k1);
    return hipGetLastError();
}

__global__ void k_fill_rows(float* dst, const float* src, int n, int rows) {
    const long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (i >= (long long)n * rows) return;
    dst[i] = src ? src[i % n] : 0.f;
}

hipError_t launch_fill_rows(float* dst, const float* src, int n, int rows, hipStream_t s) {
    const long long total = (long long)n * rows;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_rows, dim3((unsigned)((total + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, s, dst, src, n, rows);
    return hipGetLastError();
}

}  // namespace wrnn
