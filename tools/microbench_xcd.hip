// Micro-benchmark for the persistent engine's exchange primitive on MI355X.
// 256 workgroups (one per CU, forced by LDS), grouped by HW_REG_XCC_ID into 8 groups.
// Each iteration every member publishes a slice (plain or sc1 stores), then a per-member flag;
// every member polls its group's 32 flags (sc1 loads), then reads all slices (sc1 loads),
// checks every value, and proceeds. Reports per-hop time and stale reads.
// Build: hipcc -O3 --offload-arch=gfx950 tools/microbench_xcd.hip -o tools/mb_xcd
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kG = 8, kM = 32, kThreads = 512;

struct Ctl {
    unsigned reg_count[8];
    unsigned total;
    unsigned abort;
    unsigned pad[6];
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_plain(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_sc1(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned now() { return (unsigned)__builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ unsigned ld_nt(const unsigned* p) { return __builtin_nontemporal_load(p); }

// MODE bits: 1 = sc1 data stores, 2 = sc1 flag store, 4 = nt flag polls (else sc1),
//            8 = nt data loads (else sc1), 16 = data loaded as 4 independent loads per thread
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_xchg(Ctl* ctl, unsigned* flags, unsigned* data,
                                                   int slice, int iters, unsigned* out) {
    constexpr bool SC1_STORE = MODE & 1, SC1_FLAG = MODE & 2, NT_POLL = MODE & 4, NT_LOAD = MODE & 8;
    extern __shared__ unsigned lds[];
    __shared__ int s_group, s_slot, s_ok;
    const int tid = threadIdx.x;
    if (tid == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        const int g = x & 7;
        const int slot = atomicAdd(&ctl->reg_count[g], 1u);
        atomicAdd(&ctl->total, 1u);
        s_group = g;
        s_slot = slot;
        // wait for everyone to register (bounded)
        const unsigned t0 = now();
        int ok = 1;
        while (ld_sc1(&ctl->total) < (unsigned)(kG * kM)) {
            __builtin_amdgcn_s_sleep(2);
            if (now() - t0 > 20000000u) { ok = 0; break; }  // 200 ms
        }
        if (ok)
            for (int i = 0; i < kG; ++i)
                if (ld_sc1(&ctl->reg_count[i]) != kM) ok = 0;
        s_ok = ok;
        out[blockIdx.x * 4 + 0] = g;
        out[blockIdx.x * 4 + 1] = slot;
    }
    __syncthreads();
    if (!s_ok) return;
    const int g = s_group, slot = s_slot;
    unsigned* gflags = flags + g * 64;           // 32 used, one line each 128 B
    unsigned* gdata = data + (size_t)g * kM * slice;
    unsigned stale = 0;
    const unsigned t_start = now();
    for (int it = 1; it <= iters; ++it) {
        // publish my slice
        for (int i = tid; i < slice; i += kThreads) {
            const unsigned v = (unsigned)(it * 1000003u + slot * 7919u + i);
            if (SC1_STORE) st_sc1(&gdata[slot * slice + i], v);
            else gdata[slot * slice + i] = v;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            if (SC1_FLAG) st_sc1(&gflags[slot], (unsigned)it);
            else st_plain(&gflags[slot], (unsigned)it);
        }
        // wait for the group
        if (tid < 64) {
            const unsigned t0 = now();
            while (true) {
                const unsigned f = tid < kM ? (NT_POLL ? ld_nt(&gflags[tid]) : ld_sc1(&gflags[tid])) : (unsigned)it;
                if (__all(f >= (unsigned)it)) break;
                if (now() - t0 > 20000000u) { atomicOr(&ctl->abort, 1u); break; }
                if (ld_sc1(&ctl->abort)) break;
            }
        }
        __syncthreads();
        if (ld_sc1(&ctl->abort)) break;
        // read everything (sc1 loads) and verify
        {
            constexpr int U = 24;  // up to 24 loads per thread in flight
            unsigned vals[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = tid + u * kThreads;
                vals[u] = 0;
                if (i < kM * slice) vals[u] = NT_LOAD ? ld_nt(&gdata[i]) : ld_sc1(&gdata[i]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = tid + u * kThreads;
                if (i < kM * slice) {
                    const int s = i / slice, j = i % slice;
                    const unsigned e = (unsigned)(it * 1000003u + s * 7919u + j);
                    if (vals[u] != e) ++stale;
                }
            }
        }
        __syncthreads();
    }
    const unsigned t_end = now();
    atomicAdd(&out[1024], stale);
    if (tid == 0) { out[blockIdx.x * 4 + 2] = t_start; out[blockIdx.x * 4 + 3] = t_end; }
}

int main() {
    Ctl* ctl;
    unsigned *flags, *data, *out;
    CK(hipMalloc(&ctl, sizeof(Ctl)));
    CK(hipMalloc(&flags, kG * 64 * 4));
    CK(hipMalloc(&data, 8 << 20));
    CK(hipMalloc(&out, 8192 * 4));
    std::vector<unsigned> h(2048);
    const int lds = 100 * 1024;
    CK(hipFuncSetAttribute((const void*)k_xchg<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipFuncSetAttribute((const void*)k_xchg<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    auto run = [&](auto kern, int mode) -> int {
        CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        for (int slice : {16, 96, 288}) {
            const int iters = 2000;
            CK(hipMemset(ctl, 0, sizeof(Ctl)));
            CK(hipMemset(flags, 0, kG * 64 * 4));
            CK(hipMemset(out, 0, 8192 * 4));
            hipLaunchKernelGGL(kern, dim3(kG * kM), dim3(kThreads), lds, 0, ctl, flags, data, slice, iters, out);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), out, 2048 * 4, hipMemcpyDeviceToHost));
            Ctl c;
            CK(hipMemcpy(&c, ctl, sizeof(Ctl), hipMemcpyDeviceToHost));
            unsigned mn = ~0u, mx = 0;
            for (int b = 0; b < 256; ++b) { mn = std::min(mn, h[b * 4 + 2]); mx = std::max(mx, h[b * 4 + 3]); }
            printf("mode %2d [data %s, flag %s, poll %s, load %s] %5d B: abort %u stale %8u | %.3f us/hop\n", mode,
                   mode & 1 ? "sc1 " : "plain", mode & 2 ? "sc1 " : "plain", mode & 4 ? "nt " : "sc1", mode & 8 ? "nt " : "sc1",
                   slice * 128, c.abort, h[1024], (mx - mn) * 0.01 / iters);
        }
        return 0;
    };
    run(k_xchg<3>, 3);    // sc1 everything, sc1 loads (batched)
    run(k_xchg<3 | 8>, 11);   // sc1 stores, nt data loads
    run(k_xchg<0 | 4 | 8>, 12);  // plain stores + plain flag, nt polls + nt loads
    run(k_xchg<2 | 8>, 10);   // plain data, sc1 flag, sc1 poll, nt data loads
    run(k_xchg<3 | 4 | 8>, 15);  // sc1 stores, nt polls, nt loads
    return 0;
}
