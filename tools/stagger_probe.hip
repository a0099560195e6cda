// Does the placement of K1's five streams (g, mmt, vec read; mmt, vec written) move
// the HBM rate? The K1-shaped probe (3 non-temporal 16-B loads + 2 stores per float4)
// over 1 GiB per stream: five separate hipMallocs, then one allocation carved with the
// streams `pad` bytes apart beyond their size (pad 0 = back to back). Prints GB/s.
// Build: hipcc --offload-arch=gfx950 -O3 tools/stagger_probe.hip -o tools/stagger_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(x[0], x[1], x[2], x[3]);
}
__device__ __forceinline__ void st_nt(float4* p, const float4& v) {
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(p));
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_3r2w(const float4* __restrict__ a, const float4* __restrict__ b,
                                              const float4* __restrict__ c, float4* __restrict__ d,
                                              float4* __restrict__ e, long long n4) {
    const long long v = (long long)blockIdx.x * 256 + threadIdx.x;
    if (v >= n4) return;
    const float4 x = ld_nt(a + v), y = ld_nt(b + v), z = ld_nt(c + v);
    st_nt(d + v, make_float4(x.x + z.x, x.y + z.y, x.z + z.z, x.w + z.w));
    st_nt(e + v, make_float4(y.x + z.x, y.y + z.y, y.z + z.z, y.w + z.w));
}

static float run(float* p[5], long long n) {
    const long long n4 = n / 4;
    hipEvent_t s, t;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&t));
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(s, 0));
        hipLaunchKernelGGL(k_3r2w, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, 0, (const float4*)p[0],
                           (const float4*)p[1], (const float4*)p[2], (float4*)p[3], (float4*)p[4], n4);
        CK(hipEventRecord(t, 0));
        CK(hipEventSynchronize(t));
        float ms;
        CK(hipEventElapsedTime(&ms, s, t));
        if (rep) best = std::min(best, ms);   // rep 0: first touch
    }
    return 20.f * (float)n / best / 1e6f;   // GB/s
}

int main() {
    const long long n = 1ll << 28;   // floats per stream: 1 GiB
    const long long maxpad = 1 << 20;
    char* base;
    CK(hipMalloc(&base, 5 * (n * 4 + maxpad)));
    CK(hipMemset(base, 0, 5 * (n * 4 + maxpad)));
    float* sep[5];
    for (int i = 0; i < 5; ++i) {
        CK(hipMalloc(&sep[i], n * sizeof(float) + maxpad));
        CK(hipMemset(sep[i], 0, n * sizeof(float) + maxpad));
    }
    const long long pads[] = {0, 4096, 8192, 12288, 2048, 65536 + 4096};
    for (int round = 0; round < 3; ++round) {
        printf("{\"round\": %d, \"layout\": \"separate\", \"GBs\": %.1f}\n", round, run(sep, n));
        for (long long pad : pads) {
            float* p[5];
            for (int i = 0; i < 5; ++i) p[i] = reinterpret_cast<float*>(base + i * (n * 4 + pad));
            printf("{\"round\": %d, \"layout\": \"one allocation\", \"pad_bytes\": %lld, \"GBs\": %.1f}\n",
                   round, pad, run(p, n));
        }
        for (long long step : {4096ll, 8192ll}) {   // separate allocations, stream i shifted by i * step
            float* p[5];
            for (int i = 0; i < 5; ++i) p[i] = reinterpret_cast<float*>(reinterpret_cast<char*>(sep[i]) + i * step);
            printf("{\"round\": %d, \"layout\": \"separate shifted\", \"step_bytes\": %lld, \"GBs\": %.1f}\n",
                   round, step, run(p, n));
        }
    }
    for (int i = 0; i < 5; ++i) CK(hipFree(sep[i]));
    CK(hipFree(base));
    return 0;
}
