// Micro-benchmark: what a kernel boundary costs the next kernel's first loads on MI355X.
// Each reader workgroup stamps s_memrealtime at start and after its loads are consumed.
//   A) read-only table re-read by consecutive launches (is it L2/MALL resident?)
//   B) buffer written by the previous kernel (cross-XCD producers), then read
//   C) f64 log / Philox cost inside one workgroup
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_lat.hip -o /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include <cmath>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_write(float* buf, int n, float v) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] = v + i;
}

// each WG reads `per_wg` floats (float4) starting at (blockIdx.x * stride) and stamps
__global__ void k_read(const float* buf, int per_wg, long long stride, uint32_t* st, float* sink) {
    uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    const float4* p = reinterpret_cast<const float4*>(buf + blockIdx.x * stride);
    float4 acc = make_float4(0, 0, 0, 0);
    for (int i = threadIdx.x; i < per_wg / 4; i += blockDim.x) {
        float4 v = p[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    float s = acc.x + acc.y + acc.z + acc.w;
    __syncthreads();
    uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { st[2 * blockIdx.x] = t0; st[2 * blockIdx.x + 1] = t1; }
    if (s == 12345.f) sink[0] = s;
}

__global__ void k_log(uint32_t* st, float* sink, int reps) {
    uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    double acc = 0;
    uint32_t x = threadIdx.x * 2654435761u + 12345u;
    for (int r = 0; r < reps; ++r) {
        x = x * 1664525u + 1013904223u;
        const double u = (2.0 * (double)(x >> 9) + 1.0) * (1.0 / 16777216.0);
        acc += -log(u);
    }
    __syncthreads();
    uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { st[0] = t0; st[1] = t1; }
    if (acc == 1.2345) sink[0] = (float)acc;
}

__global__ void k_logf(uint32_t* st, float* sink, int reps) {
    uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    float acc = 0;
    uint32_t x = threadIdx.x * 2654435761u + 12345u;
    for (int r = 0; r < reps; ++r) {
        x = x * 1664525u + 1013904223u;
        const float u = ((float)(x >> 9) + 0.5f) * (1.0f / 8388608.0f);
        acc += -logf(u);
    }
    __syncthreads();
    uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { st[0] = t0; st[1] = t1; }
    if (acc == 1.2345f) sink[0] = acc;
}

__global__ void k_empty(uint32_t* st) {
    if (threadIdx.x == 0) { uint32_t t = (uint32_t)__builtin_amdgcn_s_memrealtime(); st[2 * blockIdx.x] = t; st[2 * blockIdx.x + 1] = t; }
}

static void report(const char* name, const std::vector<uint32_t>& st, int nwg) {
    std::vector<double> d;
    uint32_t mn = st[0];
    for (int w = 0; w < nwg; ++w) mn = std::min(mn, st[2 * w]);
    double mx = 0;
    for (int w = 0; w < nwg; ++w) { d.push_back((st[2 * w + 1] - st[2 * w]) * 0.01); mx = std::max(mx, (st[2 * w + 1] - mn) * 0.01); }
    std::sort(d.begin(), d.end());
    printf("%-48s wg=%4d per-WG load time med %.2f us max %.2f us; first-start->last-end %.2f us\n", name, nwg, d[d.size() / 2], d.back(), mx);
}

int main() {
    const int NB = 64 << 20;  // 256 MB buffer
    float *buf, *tab, *sink;
    uint32_t* st;
    CK(hipMalloc(&buf, NB * 4));
    CK(hipMalloc(&tab, 16 << 20));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&st, 1 << 20));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<uint32_t> h(8192);
    auto run_read = [&](const char* name, const float* p, int nwg, int per_wg, long long stride) {
        hipLaunchKernelGGL(k_read, dim3(nwg), dim3(256), 0, s, p, per_wg, stride, st, sink);
        hipStreamSynchronize(s);
        hipMemcpy(h.data(), st, nwg * 8, hipMemcpyDeviceToHost);
        report(name, h, nwg);
    };
    // A: weights-like table: 256 WGs x 24 KB distinct slices, launched repeatedly
    hipLaunchKernelGGL(k_write, dim3(1024), dim3(256), 0, s, tab, 4 << 20, 1.f);
    for (int i = 0; i < 4; ++i) run_read("A read-only table 256x24KB (repeat)", tab, 256, 6144, 6144);
    // A2: same but with an unrelated kernel in between
    for (int i = 0; i < 2; ++i) {
        hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, st + 4096);
        run_read("A2 table after an empty kernel", tab, 256, 6144, 6144);
    }
    // B: 36 KB vector written by 128 WGs of the previous kernel, read by every WG
    for (int i = 0; i < 3; ++i) {
        hipLaunchKernelGGL(k_write, dim3(128), dim3(256), 0, s, buf, 9216, (float)i);
        run_read("B 36KB just written, read by 256 WGs", buf, 256, 9216, 0);
    }
    for (int i = 0; i < 2; ++i) run_read("B2 36KB read again (no write between)", buf, 256, 9216, 0);
    // B3: 36 KB just written, read by 18 WGs (sampler-like)
    for (int i = 0; i < 2; ++i) {
        hipLaunchKernelGGL(k_write, dim3(128), dim3(256), 0, s, buf, 9216, (float)i);
        run_read("B3 2KB/row just written, 18 WGs read own row", buf, 18, 512, 512);
    }
    // D: cold HBM: far apart slices of the 256 MB buffer
    run_read("D cold 256 WGs x 24KB far apart", buf + (8 << 20), 256, 6144, 1 << 16);
    // C: f64 log vs f32 log, 256 threads, 2 / 16 per thread
    for (int reps : {2, 16}) {
        hipLaunchKernelGGL(k_log, dim3(1), dim3(256), 0, s, st, sink, reps);
        hipStreamSynchronize(s);
        hipMemcpy(h.data(), st, 8, hipMemcpyDeviceToHost);
        printf("C f64 -log(u) x%2d per thread: %.2f us\n", reps, (h[1] - h[0]) * 0.01);
        hipLaunchKernelGGL(k_logf, dim3(1), dim3(256), 0, s, st, sink, reps);
        hipStreamSynchronize(s);
        hipMemcpy(h.data(), st, 8, hipMemcpyDeviceToHost);
        printf("C f32 -logf(u) x%2d per thread: %.2f us\n", reps, (h[1] - h[0]) * 0.01);
    }
    // E: back-to-back empty kernels in a graph: boundary cost
    {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s, st + 16 * i);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int it = 0; it < 3; ++it) {
            hipEventRecord(e0, s);
            hipGraphLaunch(ge, s);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("E graph of 100 empty 256-WG kernels: %.2f us per kernel\n", ms * 1000 / 100);
        }
    }
    return 0;
}
