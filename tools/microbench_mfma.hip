// Microbenchmark + layout probe for the persistent kernels' matrix-vector stages on gfx950.
//
// 1. Probes the operand / result layout of v_mfma_f32_4x4x1f32 (16 blocks of 4x4x1).
// 2. Times one stage-A-shaped product (48 gate rows x 512 k of one workgroup slot, NR = 3 fold
//    rows staged in LDS) on the four critical waves, three ways:
//      VALU  : the current kernels_persist.hip scheme (v_pk_fma_f32 + DPP row16 reduction)
//      MFMA  : 4x4x1 blocks = 16 k-slices of one 4-output quad, 3 quads per wave, B operand from
//              one ds_read_b128 per 4 MFMAs, DPP + permlane-swap reduction over the 16 blocks
//    each alone (waves 4-7 idle) and beside a copy of itself in waves 4-7 (the W_hh1 partner).
//    Results of both are compared (fp32 tolerance; the summation orders differ).
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/mb_mfma tools/microbench_mfma.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

__global__ void k_probe(float* out) {
    const int l = threadIdx.x;
    v4f c = {0.f, 0.f, 0.f, 0.f};
    // pass 1: A = lane + 1, B = 1 -> D shows where A_b[i] lives
    v4f d1 = __builtin_amdgcn_mfma_f32_4x4x1f32((float)(l + 1), 1.0f, c, 0, 0, 0);
    // pass 2: A = 1, B = lane + 1 -> where B_b[j] lives
    v4f d2 = __builtin_amdgcn_mfma_f32_4x4x1f32(1.0f, (float)(l + 1), c, 0, 0, 0);
    for (int v = 0; v < 4; ++v) {
        out[v * 64 + l] = d1[v];
        out[256 + v * 64 + l] = d2[v];
    }
}

constexpr int K = 512, NR = 3, XS = 528;  // x row stride (floats), 528 = 16 mod 64 banks

template <int CTRL>
__device__ __forceinline__ float pdpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row16_sum(float v) {
    v += pdpp<0xB1>(v);
    v += pdpp<0x4E>(v);
    v += pdpp<0x124>(v);
    v += pdpp<0x128>(v);
    return v;
}
__device__ __forceinline__ void dot4(v2f& acc, const float4 w, const float4 x) {
    acc = __builtin_elementwise_fma((v2f){w.x, w.y}, (v2f){x.x, x.y}, acc);
    acc = __builtin_elementwise_fma((v2f){w.z, w.w}, (v2f){x.z, x.w}, acc);
}
// sum over lanes l, l^16, l^32, l^48 and within the 16-lane row over l%4-equal lanes:
// every lane receives the total of its column (l % 4)
__device__ __forceinline__ float blocks16_sum(float v) {
    v += pdpp<0x124>(v);  // row_ror 4
    v += pdpp<0x128>(v);  // row_ror 8
    {
        auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    {
        auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
        v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
    }
    return v;
}

// W: [48][K] (row o = gate j * 16 + unit ul), X: [NR][K]. mode 0 VALU, 1 MFMA; partner: waves
// 4-7 run the same body; out: [NR][48] results of workgroup 0; cyc: cycles per iteration.
template <int MODE, int NCH = 1>
__global__ __launch_bounds__(512, 1) void k_stage(const float* W, const float* X, float* out,
                                                  unsigned* cyc, int iters, int partner) {
    __shared__ __attribute__((aligned(16))) float xs[NR * XS];
    __shared__ float res[NR * 48];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < NR * K; i += 512) xs[(i / K) * XS + i % K] = X[i];
    const bool active = MODE == 2 || wave < 4 || partner;
    const int wq = wave & 3;
    // ---- weights to registers
    float4 wv[24];   // VALU: og = tid / 16 (unit og % 16), kc = tid % 16, 3 gates x 8 float4
    float4 w8[12];   // VALU8: unit u8 = tid / 32, kc8 = tid % 32, 3 gates x 4 float4
    const int u8 = tid >> 5, kc8 = tid & 31;
    float wm[96];    // MFMA: quad j (gate j, units 4 wq .. 4 wq + 3), group g, c
    const int og = (tid >> 4) & 15, kc = tid & 15;
    const int b = lane >> 2, ii = lane & 3;
    if (MODE == 2) {
        for (int j = 0; j < 3; ++j)
            for (int q = 0; q < 4; ++q) {
                const float* p = W + (size_t)(j * 16 + u8) * K + 4 * (32 * q + kc8);
                w8[j * 4 + q] = make_float4(p[0], p[1], p[2], p[3]);
            }
    } else if (MODE == 0) {
        for (int j = 0; j < 3; ++j)
            for (int q = 0; q < 8; ++q) {
                const float* p = W + (size_t)(j * 16 + og) * K + 4 * (16 * q + kc);
                wv[j * 8 + q] = make_float4(p[0], p[1], p[2], p[3]);
            }
    } else {
        for (int j = 0; j < 3; ++j)
            for (int g = 0; g < 8; ++g)
                for (int c = 0; c < 4; ++c)
                    wm[j * 32 + g * 4 + c] = W[(size_t)(j * 16 + 4 * wq + ii) * K + 64 * g + 4 * b + c];
    }
    __syncthreads();
    float sink = 0.f;
    unsigned t0 = 0, t1 = 0;
    for (int it = 0; it < iters; ++it) {
        if (it == 1) t0 = (unsigned)__builtin_amdgcn_s_memtime();
        if (active) {
            if (wave < 4) __builtin_amdgcn_s_setprio(2);
            if (MODE == 2) {
                const float4* X4 = reinterpret_cast<const float4*>(xs);
                float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    v2f acc[3] = {(v2f){0.f, 0.f}, (v2f){0.f, 0.f}, (v2f){0.f, 0.f}};
                    float4 xq[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) xq[q] = X4[r * (XS / 4) + 32 * q + kc8];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int j = 0; j < 3; ++j) dot4(acc[j], w8[j * 4 + q], xq[q]);
                    float t[3];
#pragma unroll
                    for (int j = 0; j < 3; ++j) {
                        float v = row16_sum(acc[j].x + acc[j].y);
                        auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
                        t[j] = __uint_as_float(p[0]) + __uint_as_float(p[1]);
                    }
                    if (kc8 == r) { s0 = t[0]; s1 = t[1]; s2 = t[2]; }
                }
                sink += s0 + s1 + s2;
                if (it == iters - 1 && kc8 < NR) {
                    res[kc8 * 48 + 0 * 16 + u8] = s0;
                    res[kc8 * 48 + 1 * 16 + u8] = s1;
                    res[kc8 * 48 + 2 * 16 + u8] = s2;
                }
            } else if (MODE == 0) {
                const float4* X4 = reinterpret_cast<const float4*>(xs);
                float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    v2f acc[3] = {(v2f){0.f, 0.f}, (v2f){0.f, 0.f}, (v2f){0.f, 0.f}};
#pragma unroll
                    for (int qb = 0; qb < 8; qb += 4) {
                        __builtin_amdgcn_sched_barrier(0);
                        float4 xq[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) xq[q] = X4[r * (XS / 4) + 16 * (qb + q) + kc];
#pragma unroll
                        for (int q = 0; q < 4; ++q)
#pragma unroll
                            for (int j = 0; j < 3; ++j) dot4(acc[j], wv[j * 8 + qb + q], xq[q]);
                    }
                    const float t0_ = row16_sum(acc[0].x + acc[0].y);
                    const float t1_ = row16_sum(acc[1].x + acc[1].y);
                    const float t2_ = row16_sum(acc[2].x + acc[2].y);
                    if (kc == r) { s0 = t0_; s1 = t1_; s2 = t2_; }
                }
                sink += s0 + s1 + s2;
                if (it == iters - 1 && wave < 4 && kc < NR) {
                    res[kc * 48 + 0 * 16 + og] = s0;
                    res[kc * 48 + 1 * 16 + og] = s1;
                    res[kc * 48 + 2 * 16 + og] = s2;
                }
            } else {
                v4f d[3][NCH];
#pragma unroll
                for (int j = 0; j < 3; ++j)
#pragma unroll
                    for (int e = 0; e < NCH; ++e) d[j][e] = (v4f){0.f, 0.f, 0.f, 0.f};
                const int r = ii < NR ? ii : 0;  // B column = fold row (lane % 4), row 3 unused
#pragma unroll
                for (int g = 0; g < 8; ++g) {
                    const float4 xb = *reinterpret_cast<const float4*>(xs + r * XS + 64 * g + 4 * b);
                    const float bx[4] = {xb.x, xb.y, xb.z, xb.w};
#pragma unroll
                    for (int c = 0; c < 4; ++c)
#pragma unroll
                        for (int j = 0; j < 3; ++j)
                            d[j][(g * 4 + c) % NCH] = __builtin_amdgcn_mfma_f32_4x4x1f32(
                                wm[j * 32 + g * 4 + c], bx[c], d[j][(g * 4 + c) % NCH], 0, 0, 0);
                }
                float s[3][4];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    v4f t = d[j][0];
#pragma unroll
                    for (int e = 1; e < NCH; ++e) t += d[j][e];
#pragma unroll
                    for (int v = 0; v < 4; ++v) s[j][v] = blocks16_sum(t[v]);
                }
                sink += s[0][0] + s[1][1] + s[2][2];
                if (it == iters - 1 && wave < 4 && b == 0 && ii < NR)
                    for (int j = 0; j < 3; ++j)
                        for (int v = 0; v < 4; ++v) res[ii * 48 + j * 16 + 4 * wq + v] = s[j][v];
            }
            __builtin_amdgcn_s_setprio(0);
        }
        __syncthreads();
    }
    t1 = (unsigned)__builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0) {
        if (tid == 0) cyc[0] = (t1 - t0) / (unsigned)(iters - 1);
        for (int i = tid; i < NR * 48; i += 512) out[i] = res[i];
        if (tid == 1) cyc[1] = __float_as_uint(sink);
    }
}

int main() {
    float* dout;
    HC(hipMalloc(&dout, 2048 * sizeof(float)));
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dout);
    std::vector<float> h(512);
    HC(hipMemcpy(h.data(), dout, 512 * sizeof(float), hipMemcpyDeviceToHost));
    std::printf("probe A=lane+1,B=1: D[v][lane] for lanes 0..19\n");
    for (int v = 0; v < 4; ++v) {
        std::printf(" v%d:", v);
        for (int l = 0; l < 20; ++l) std::printf(" %3.0f", h[v * 64 + l]);
        std::printf("\n");
    }
    std::printf("probe A=1,B=lane+1\n");
    for (int v = 0; v < 4; ++v) {
        std::printf(" v%d:", v);
        for (int l = 0; l < 20; ++l) std::printf(" %3.0f", h[256 + v * 64 + l]);
        std::printf("\n");
    }
    // stage benchmark
    std::vector<float> W(48 * K), X(NR * K);
    srand(1);
    for (auto& w : W) w = (float)rand() / (float)RAND_MAX - 0.5f;
    for (auto& x : X) x = (float)rand() / (float)RAND_MAX - 0.5f;
    float *dW, *dX;
    unsigned* dc;
    HC(hipMalloc(&dW, W.size() * 4));
    HC(hipMalloc(&dX, X.size() * 4));
    HC(hipMalloc(&dc, 16));
    HC(hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice));
    HC(hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice));
    std::vector<double> ref(NR * 48);
    for (int r = 0; r < NR; ++r)
        for (int o = 0; o < 48; ++o) {
            double s = 0;
            for (int k = 0; k < K; ++k) s += (double)W[o * K + k] * X[r * K + k];
            ref[r * 48 + o] = s;
        }
    const int iters = 2000;
    for (int mode = 0; mode < 5; ++mode)
        for (int partner = 0; partner < 2; ++partner) {
            if (mode == 4) hipLaunchKernelGGL(k_stage<2>, dim3(256), dim3(512), 0, 0, dW, dX, dout, dc, iters, partner);
            else if (mode == 0) hipLaunchKernelGGL(k_stage<0>, dim3(256), dim3(512), 0, 0, dW, dX, dout, dc, iters, partner);
            else if (mode == 1) hipLaunchKernelGGL((k_stage<1, 1>), dim3(256), dim3(512), 0, 0, dW, dX, dout, dc, iters, partner);
            else if (mode == 2) hipLaunchKernelGGL((k_stage<1, 2>), dim3(256), dim3(512), 0, 0, dW, dX, dout, dc, iters, partner);
            else hipLaunchKernelGGL((k_stage<1, 4>), dim3(256), dim3(512), 0, 0, dW, dX, dout, dc, iters, partner);
            HC(hipGetLastError());
            HC(hipDeviceSynchronize());
            unsigned c[2];
            std::vector<float> o(NR * 48);
            HC(hipMemcpy(c, dc, 8, hipMemcpyDeviceToHost));
            HC(hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost));
            double err = 0;
            for (int i = 0; i < NR * 48; ++i) err = std::fmax(err, std::fabs(o[i] - ref[i]));
            std::printf("%s chains/quad=%d partner=%d: %u cycles / stage (incl. barrier), max |err| vs f64 %.3g\n",
                        mode == 4 ? "VALU 8 waves" : mode ? "MFMA 4x4x1" : "VALU pk_fma", mode == 3 ? 4 : mode, partner, c[0], err);
        }
    return 0;
}
