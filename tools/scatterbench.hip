// Scattered-store throughput on this MI355X: what the decompress's W*k scattered
// writes (and the sparse re-zero) are bound by. M random distinct 128-B lines of a
// 4 GB buffer get either one 4-B store, one 64-B store (4 lanes x 16 B) or a full
// 128-B line (8 lanes x 16 B). Prints the ms per variant.
// Build: hipcc --offload-arch=gfx950 -O3 tools/scatterbench.hip -o tools/scatterbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_store4(float* buf, const unsigned* lines, int m) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) buf[(size_t)lines[i] * 32 + 5] = 1.f;
}
// G lanes per line, 16 B each (G = 4: 64 B, G = 8: 128 B)
template <int G>
__global__ void k_storeline(float4* buf, const unsigned* lines, int m) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = i / G, part = i % G;
    if (l < m) buf[(size_t)lines[l] * 8 + part] = make_float4(1.f, 0.f, 0.f, 0.f);
}

int main() {
    const size_t n = 1ull << 30;              // floats: 4 GB
    const size_t nlines = n / 32;
    float* buf;
    CK(hipMalloc(&buf, n * sizeof(float)));
    CK(hipMemset(buf, 0, n * sizeof(float)));
    for (int m : {1 << 20, 8 << 20}) {
        std::vector<unsigned> h(m);
        std::mt19937_64 rng(1);
        std::vector<unsigned char> used(nlines, 0);
        for (int i = 0; i < m;) {
            const unsigned l = (unsigned)(rng() % nlines);
            if (!used[l]) { used[l] = 1; h[i++] = l; }
        }
        std::sort(h.begin(), h.end());   // the decompress writes in index order
        unsigned* d;
        CK(hipMalloc(&d, m * sizeof(unsigned)));
        CK(hipMemcpy(d, h.data(), m * sizeof(unsigned), hipMemcpyHostToDevice));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        float ms[3];
        for (int v = 0; v < 3; ++v) {
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(a, 0));
                if (v == 0) hipLaunchKernelGGL(k_store4, dim3((m + 255) / 256), dim3(256), 0, 0, buf, d, m);
                if (v == 1) hipLaunchKernelGGL(k_storeline<4>, dim3((4 * m + 255) / 256), dim3(256), 0, 0,
                                               reinterpret_cast<float4*>(buf), d, m);
                if (v == 2) hipLaunchKernelGGL(k_storeline<8>, dim3((8 * m + 255) / 256), dim3(256), 0, 0,
                                               reinterpret_cast<float4*>(buf), d, m);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                best = std::min(best, t);
            }
            ms[v] = best;
        }
        printf("{\"lines\": %d, \"store4_ms\": %.4f, \"store64B_ms\": %.4f, \"store128B_ms\": %.4f}\n", m, ms[0], ms[1],
               ms[2]);
        CK(hipFree(d));
    }
    CK(hipFree(buf));
    return 0;
}
