// GEMM-shaped precompute of the vocoder: the MelResNet convolutions of the upsample network
// (reference vocoder/models/fatchord_version.py:9-44) and the conditioning products that the
// recurrence consumes every step (the aux/mel parts of I, rnn2/rnn3, fc1..fc3 input concats,
// fatchord_version.py:198-211). These are the dense contractions of the path, so they run on
// the fp32 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32, an fma chain in k order).
//
// D[m][n] = sum_k A(m,k) B(k,n): 64x64 workgroup tile, 4 waves of 32x32, BK = 16 staged in LDS
// as [k][m] / [k][n] so each MFMA operand read is one conflict-free 32-lane row.
// Also here: the stretch + box-conv stencils of the mel upsampler (fatchord_version.py:47-85).
#include "wrnn_kernels.h"

namespace wrnn {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int kGemmWavesPerSimd = 3;  // waves per SIMD the GEMM is compiled for
constexpr int kGemmWideNT = 4;        // 64-wide column tiles per workgroup for wide outputs (P1)

// A(m, .) of one row as two strided segments: k < ksplit reads p0[o0 + k * s0], the rest
// p1[o1 + k * s1] (o1 may be negative: it is only ever used with k >= ksplit). The row's
// index math (the fold_with_overlap position, its frame) runs once per thread, not per k.
struct ARow {
    const float *p0, *p1;
    long o0, o1;
    int s0, s1, ksplit;
    bool zero;
};

// AK = GemmA::kind as a template argument: one straight-line row setup per kernel (a runtime
// switch over the kinds here was mis-structured by the compiler: the frame-A path lost p0).
template <int AK>
__device__ __forceinline__ ARow a_row(const GemmA& a, int m, int M) {
    ARow r{};
    r.zero = m >= M;
    if constexpr (AK == 0) {
        r.p0 = r.p1 = a.p;
        r.o0 = r.o1 = (long)m * a.ld;
        r.s0 = r.s1 = 1;
        r.ksplit = 1 << 30;
    } else if constexpr (AK == 1) {  // cI: [mel_up(p) (n_mel) | aux(p // hop)[r_off : r_off + n_aux]]
        // fold-major rows (m = fold * S + step, M = S * Bu): the 64 rows of a tile are
        // consecutive positions of one or two folds, so each k reads whole cache lines
        const int S = M / a.Bu, f = m / S, t = m - f * S;
        const int p = (a.f0 + f) * a.tpo + t;  // fold_with_overlap position
        r.zero |= p >= a.L;                            // zero tail pad
        r.p0 = a.mel;
        r.o0 = p;
        r.s0 = a.ldm;
        r.p1 = a.R;
        r.o1 = (long)(a.r_off - a.n_mel) * a.ldr + p / a.hop;
        r.s1 = a.ldr;
        r.ksplit = a.n_mel;
    } else {  // frame-A: slot 0 is the zero frame; slot f+1 = frame f
        r.zero |= m == 0;
        r.p0 = r.p1 = a.R;
        r.o0 = r.o1 = (long)a.r_off * a.ldr + (m - 1);
        r.s0 = r.s1 = a.ldr;
        r.ksplit = 1 << 30;
    }
    return r;
}

__device__ __forceinline__ float load_a(const ARow& r, int k, int K) {
    if (r.zero || k >= K) return 0.f;
    return k < r.ksplit ? r.p0[r.o0 + (long)k * r.s0] : r.p1[r.o1 + (long)k * r.s1];
}

__device__ __forceinline__ float load_b(const GemmB& b, int k, int n) {
    if (b.kind == 0) return b.p[(size_t)k * b.ld + n];
    // im2col of the zero-padded mel (pad_tensor(.., pad, 'both'), fatchord_version.py:171)
    const int ci = k / b.ksz, kk = k % b.ksz;
    const int i = n + kk - b.pad;
    return (i >= 0 && i < b.T) ? b.p[(size_t)ci * b.T + i] : 0.f;
}

__device__ __forceinline__ void store_ep(const GemmEp& e, int m, int n, float acc) {
    float v;
    switch (e.kind) {
        case 0:
            v = acc + e.bias[n];
            break;
        case 1:
            v = acc + e.bias[m];
            break;
        default: {  // kind 2 (kind 3, the folded rows, is stored by k_gemm itself)
            // eval BatchNorm as torch CPU: x * (w / sqrt(var + eps)) + (b - mean * alpha)
            v = fmaf(acc, e.alpha[m], e.beta[m]);
            if (e.relu) v = v > 0.f ? v : 0.f;
            if (e.res) v = v + e.res[(size_t)m * e.ld + n];
            break;
        }
    }
    e.D[(size_t)m * e.ld + n] = v;
}

// NT 64-wide column tiles per workgroup share one staged A tile (the gathered conditioning
// rows are read once per k step, not once per column tile). The next k step's operands are
// fetched into registers while the matrix cores work on the current one.
// BK = k depth staged per step: 16 for the large conditioning GEMMs (K = 111), 64 for the small
// launch-latency-bound MelResNet GEMMs (two to seven global round trips per tile instead of 8-25;
// the k order of the MFMA chain is the same, so are the results).
template <int NT, int AK, int BK>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kGemmWavesPerSimd))) void k_gemm(int M, int N, int K, GemmA A, GemmB B,
                                                   GemmEp E) {
    __shared__ float As[BK][64];
    __shared__ float Bs[BK][64 * NT];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv & 1, wn = wv >> 1;
    // XCD-aware tile order: workgroup L runs on XCD L % 8; the column tiles of one row tile
    // are consecutive workgroups of one XCD, so its L2 serves their shared A rows
    const int n_tiles = (N + 64 * NT - 1) / (64 * NT), m_tiles = (M + 63) / 64;
    const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
    const int m_tile = (local / n_tiles) * 8 + xcd, n_tile = local % n_tiles;
    if (m_tile >= m_tiles) return;  // the row-tile count is padded to a multiple of 8
    const int m0 = m_tile * 64, n0 = n_tile * 64 * NT;
    // this thread stages A(m0 + (tid & 63), k0 + (tid >> 6) + 4 i), i < 4
    const ARow ar = a_row<AK>(A, m0 + (tid & 63), M);
    float ra[BK / 4], rb[BK / 4 * NT];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int i = 0; i < BK / 4; ++i) ra[i] = load_a(ar, k0 + (tid >> 6) + 4 * i, K);
#pragma unroll
        for (int i = 0; i < BK / 4 * NT; ++i) {
            const int e = tid + i * kThreads;
            const int n = n0 + e % (64 * NT), k = k0 + e / (64 * NT);
            rb[i] = (n < N && k < K) ? load_b(B, k, n) : 0.f;
        }
    };
    floatx16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    fetch(0);
    for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
        for (int i = 0; i < BK / 4; ++i) As[(tid >> 6) + 4 * i][tid & 63] = ra[i];
#pragma unroll
        for (int i = 0; i < BK / 4 * NT; ++i) {
            const int e = tid + i * kThreads;
            Bs[e / (64 * NT)][e % (64 * NT)] = rb[i];
        }
        __syncthreads();
        if (k0 + BK < K) fetch(k0 + BK);
#pragma unroll
        for (int kp = 0; kp < BK / 2; ++kp) {
            const float av = As[2 * kp + (lane >> 5)][wm * 32 + (lane & 31)];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float bv = Bs[2 * kp + (lane >> 5)][64 * t + wn * 32 + (lane & 31)];
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[t], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // C/D map (32x32, 16 regs): col = lane & 31, row = 8*(r>>2) + 4*(lane>>5) + (r&3)
    if (E.kind == 3) {  // folded rows: the row index once per r, the bias once per tile
        const int S = M / E.Bu;  // fold-major m = fold * S + step, as the kind-1 A rows
        float bias[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int n = n0 + 64 * t + wn * 32 + (lane & 31);
            bias[t] = n < N ? E.bias[n] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
            if (m >= M) continue;
            const int f = m / S, t = m - f * S;
            float* D = E.D + ((size_t)t * E.Btot + E.row0 + f) * E.ld;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int n = n0 + 64 * t + wn * 32 + (lane & 31);
                if (n < N) D[n] = acc[t][r] + bias[t];
            }
        }
        return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int i = 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
            const int j = lane & 31;
            const int m = m0 + wm * 32 + i, n = n0 + 64 * t + wn * 32 + j;
            if (m < M && n < N) store_ep(E, m, n, acc[t][r]);
        }
}

template <int NT, int BK>
static void launch_nt(dim3 grid, int M, int N, int K, const GemmA& a, const GemmB& b,
                      const GemmEp& e, hipStream_t s) {
    if (a.kind == 0)
        hipLaunchKernelGGL((k_gemm<NT, 0, BK>), grid, dim3(kThreads), 0, s, M, N, K, a, b, e);
    else if (a.kind == 1)
        hipLaunchKernelGGL((k_gemm<NT, 1, BK>), grid, dim3(kThreads), 0, s, M, N, K, a, b, e);
    else
        hipLaunchKernelGGL((k_gemm<NT, 2, BK>), grid, dim3(kThreads), 0, s, M, N, K, a, b, e);
}

hipError_t launch_gemm(int M, int N, int K, const GemmA& a, const GemmB& b, const GemmEp& e,
                       hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (a.kind < 0 || a.kind > 2) return hipErrorInvalidValue;
    const int m_tiles8 = ((M + 63) / 64 + 7) / 8 * 8;  // k_gemm's XCD-aware tile order
    if (N >= 1024)  // wide outputs (P1: 3H / 4H columns): 4 column tiles per workgroup
        launch_nt<kGemmWideNT, 16>(
            dim3(m_tiles8 * ((N + 64 * kGemmWideNT - 1) / (64 * kGemmWideNT))), M, N,
            K, a, b, e, s);
    else if ((M + 63) / 64 * ((N + 63) / 64) <= 256 && K >= 64)
        // fewer tiles than CUs (MelResNet: M = 128 channels, N = frames): latency-bound, so
        // stage k 64 deep (one global round trip per 64 k instead of per 16)
        launch_nt<1, 64>(dim3(m_tiles8 * ((N + 63) / 64)), M, N, K, a, b, e, s);
    else
        launch_nt<1, 16>(dim3(m_tiles8 * ((N + 63) / 64)), M, N, K, a, b, e, s);
    return hipGetLastError();
}

// Stretch2d(s, 1) followed by Conv2d(1, 1, (1, 2s+1), padding (0, s)), per mel channel:
// out(c, o) = sum_d w[d] * in_str(c, o + d - s), in_str(c, i) = in(c, i / s) for
// 0 <= i < W_in * s, else 0; in(c, i) = src[c][i - in_pad] inside [in_pad, in_pad + T_in).
__global__ __launch_bounds__(kThreads) void k_mel_stencil(const float* in, int in_pad, int T_in,
                                                          int W_in, float* out, int s,
                                                          const float* w, int out_lo,
                                                          int out_len, int ld_out) {
    const int oo = blockIdx.x * kThreads + threadIdx.x;
    const int c = blockIdx.y;
    if (oo >= out_len) return;
    const int o = out_lo + oo;
    const int W_out = W_in * s;
    const float* src = in + (size_t)c * T_in;
    float acc = 0.f;
    // taps in d order (the same fma chain); the stretched index i / s is advanced
    // incrementally instead of divided per tap (one division per output)
    int d = 0, i = o - s;
    if (i < 0) {
        d = -i;
        i = 0;
    }
    int q = i / s, r = i - q * s;
    for (; d <= 2 * s && i < W_out; ++d, ++i) {
        const int si = q - in_pad;
        const float v = (si >= 0 && si < T_in) ? src[si] : 0.f;
        acc = fmaf(w[d], v, acc);
        if (++r == s) {
            r = 0;
            ++q;
        }
    }
    out[(size_t)c * ld_out + oo] = acc;
}

hipError_t launch_mel_stencil(const float* in, int in_pad, int T_in, int W_in, float* out,
                              int scale, const float* w, int c, int out_lo, int out_len,
                              int ld_out, hipStream_t s) {
    if (out_len <= 0) return hipSuccess;
    dim3 grid((out_len + kThreads - 1) / kThreads, c);
    hipLaunchKernelGGL(k_mel_stencil, grid, dim3(kThreads), 0, s, in, in_pad, T_in, W_in, out,
                       scale, w, out_lo, out_len, ld_out);
    return hipGetLastError();
}

// Per-frame P1 expansion (launch_p1_expand, wrnn_kernels.h). A thread owns one float4 column
// chunk of one fold row over a run of kP1Run consecutive steps: the five frame projections
// around the current frame and its aux term stay in registers while the run stays inside one
// frame (hop steps), so an output float4 costs one store and ~6 / kP1Run loads. The phase taps
// are uniform over the workgroup (scalar loads). Output: one coalesced 1-KiB store per wave.
constexpr int kP1Run = 64;
__global__ __launch_bounds__(kThreads) void k_p1_expand(float4* __restrict__ P1, int Btot,
                                                        int row0, int f0, int S, int tpo, int L, int hop,
                                                        int T, int nq, const float4* __restrict__ q,
                                                        const float4* __restrict__ a,
                                                        const float* __restrict__ taps) {
    const int c = blockIdx.x * kThreads + threadIdx.x;
    const int fo = blockIdx.y, t0 = blockIdx.z * kP1Run;
    if (c >= nq) return;
    const int t1 = t0 + kP1Run < S ? t0 + kP1Run : S;
    const float4 z4 = {0.f, 0.f, 0.f, 0.f};
    float4 r[5], av = z4;
    int fc = -2;  // frame of the operands in registers (-1: the zero tail pad)
    for (int t = t0; t < t1; ++t) {
        const int p = (f0 + fo) * tpo + t;  // fold_with_overlap position
        const int f = p < L ? p / hop : -1;
        if (f != fc) {
            fc = f;
            if (f < 0) {
                av = a[c];  // zero frame: bias only
            } else {
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    const int j = f - 2 + k;
                    r[k] = (j >= 0 && j < T) ? q[(size_t)(j + 1) * nq + c] : z4;
                }
                av = a[(size_t)(f + 1) * nq + c];
            }
        }
        float4 v = av;
        if (f >= 0) {
            const float* K = taps + (size_t)(p - f * hop) * 8;
            float4 m = z4;
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                m.x = fmaf(K[k], r[k].x, m.x);
                m.y = fmaf(K[k], r[k].y, m.y);
                m.z = fmaf(K[k], r[k].z, m.z);
                m.w = fmaf(K[k], r[k].w, m.w);
            }
            v.x = m.x + av.x;
            v.y = m.y + av.y;
            v.z = m.z + av.z;
            v.w = m.w + av.w;
        }
        P1[((size_t)t * Btot + row0 + fo) * nq + c] = v;
    }
}

hipError_t launch_p1_expand(float* P1, int Btot, int row0, int Bu, int f0, int S, int tpo, int L,
                            int hop, int T, int nq, const float* q, const float* a, const float* taps,
                            hipStream_t s) {
    if (Bu <= 0 || S <= 0 || nq <= 0) return hipSuccess;
    if (hop <= 0 || T <= 0 || Bu > 65535) return hipErrorInvalidValue;
    dim3 grid((nq + kThreads - 1) / kThreads, Bu, (S + kP1Run - 1) / kP1Run);
    hipLaunchKernelGGL(k_p1_expand, grid, dim3(kThreads), 0, s, reinterpret_cast<float4*>(P1), Btot,
                       row0, f0, S, tpo, L, hop, T, nq, reinterpret_cast<const float4*>(q),
                       reinterpret_cast<const float4*>(a), taps);
    return hipGetLastError();
}

}  // namespace wrnn
