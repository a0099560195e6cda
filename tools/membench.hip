// HBM streaming ceilings on this MI355X for the access mixes of the DGC kernels:
//   copy (1R1W), read-only reduce (select pass), write-only fill (decompress),
//   3R2W momentum/velocity update (K1) in several code shapes.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld(const float4* p) {
    if (NT) {
        f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        return make_float4(x[0], x[1], x[2], x[3]);
    }
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(float4* p, float4 v) {
    if (NT) {
        f4v x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(p));
    } else *p = v;
}

__device__ __forceinline__ void upd(const float4& g, float4& m, float4& v, float mom) {
    m.x = __fmul_rn(__fadd_rn(m.x, g.x), mom); v.x = __fadd_rn(__fadd_rn(v.x, m.x), g.x);
    m.y = __fmul_rn(__fadd_rn(m.y, g.y), mom); v.y = __fadd_rn(__fadd_rn(v.y, m.y), g.y);
    m.z = __fmul_rn(__fadd_rn(m.z, g.z), mom); v.z = __fadd_rn(__fadd_rn(v.z, m.z), g.z);
    m.w = __fmul_rn(__fadd_rn(m.w, g.w), mom); v.w = __fadd_rn(__fadd_rn(v.w, m.w), g.w);
}

// grid-stride, U float4 per thread per iteration (strided by G)
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k3r2w(const float4* __restrict__ g, float4* __restrict__ m,
                                            float4* __restrict__ v, long n4, float mom) {
    const long G = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * G < n4; i += U * G) {
        float4 a[U], b[U], c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { a[u] = ld<NTL>(g + i + u * G); b[u] = ld<NTL>(m + i + u * G); c[u] = ld<NTL>(v + i + u * G); }
#pragma unroll
        for (int u = 0; u < U; ++u) { upd(a[u], b[u], c[u], mom); st<NTS>(m + i + u * G, b[u]); st<NTS>(v + i + u * G, c[u]); }
    }
    for (; i < n4; i += G) {
        float4 a = ld<NTL>(g + i), b = ld<NTL>(m + i), c = ld<NTL>(v + i);
        upd(a, b, c, mom); st<NTS>(m + i, b); st<NTS>(v + i, c);
    }
}

// block-contiguous chunks: each block owns CH float4 (no grid stride)
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k3r2w_chunk(const float4* __restrict__ g, float4* __restrict__ m,
                                                  float4* __restrict__ v, long n4, float mom) {
    const long base = (long)blockIdx.x * 256 * U;
    float4 a[U], b[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256 + threadIdx.x; if (i < n4) { a[u] = ld<NTL>(g + i); b[u] = ld<NTL>(m + i); c[u] = ld<NTL>(v + i); } }
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256 + threadIdx.x; if (i < n4) { upd(a[u], b[u], c[u], mom); st<NTS>(m + i, b[u]); st<NTS>(v + i, c[u]); } }
}

// 3 reads, 3 writes: the gradient chunk is zeroed after it is read (in-place decompress target)
template <int U, bool NT>
__global__ void __launch_bounds__(256) k3r3w_chunk(float4* __restrict__ g, float4* __restrict__ m,
                                                  float4* __restrict__ v, long n4, float mom) {
    const long base = (long)blockIdx.x * 256 * U;
    float4 a[U], b[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256 + threadIdx.x; if (i < n4) { a[u] = ld<NT>(g + i); b[u] = ld<NT>(m + i); c[u] = ld<NT>(v + i); } }
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256 + threadIdx.x; if (i < n4) { upd(a[u], b[u], c[u], mom); st<NT>(m + i, b[u]); st<NT>(v + i, c[u]); st<NT>(g + i, make_float4(0, 0, 0, 0)); } }
}

// one-shot fill: each block owns U*256 float4
template <int U, bool NT>
__global__ void __launch_bounds__(256) kfill_chunk(float4* __restrict__ a, long n4) {
    const long base = (long)blockIdx.x * 256 * U;
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = base + u * 256 + threadIdx.x; if (i < n4) st<NT>(a + i, make_float4(0, 0, 0, 0)); }
}

template <bool NT>
__global__ void __launch_bounds__(256) kcopy(const float4* __restrict__ a, float4* __restrict__ b, long n4) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) st<NT>(b + i, ld<NT>(a + i));
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) kread(const float4* __restrict__ a, long n4, float t, unsigned* out) {
    const long G = (long)gridDim.x * 256;
    unsigned c = 0;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * G < n4; i += U * G) {
        float4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = ld<NT>(a + i + u * G);
#pragma unroll
        for (int u = 0; u < U; ++u) c += (fabsf(x[u].x) >= t) + (fabsf(x[u].y) >= t) + (fabsf(x[u].z) >= t) + (fabsf(x[u].w) >= t);
    }
    for (; i < n4; i += G) { float4 x = ld<NT>(a + i); c += (fabsf(x.x) >= t) + (fabsf(x.w) >= t); }
    if (c == 0xFFFFFFFF) out[0] = c;
}

template <bool NT>
__global__ void __launch_bounds__(256) kfill(float4* __restrict__ a, long n4) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) st<NT>(a + i, make_float4(0, 0, 0, 0));
}

template <class F>
static float timeit(F f, int reps) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000000L;
    const long n4 = n / 4;
    float *g, *m, *v; unsigned* o;
    CK(hipMalloc(&g, n * 4)); CK(hipMalloc(&m, n * 4)); CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&o, 64));
    CK(hipMemset(g, 0x3c, n * 4)); CK(hipMemset(m, 0x3c, n * 4)); CK(hipMemset(v, 0x3c, n * 4));
    auto G4 = (const float4*)g; auto M4 = (float4*)m; auto V4 = (float4*)v;
    const int reps = 10;
    auto rep = [&](const char* name, double bytes, float ms) { printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9); fflush(stdout); };
    const bool chunk_only = argc > 2 && argv[2][0] == 'c';
    for (int U : {1, 2, 4}) {
        long blocks = (n4 + 256L * U - 1) / (256L * U);
        char nm[96];
        auto G4w = (float4*)g;
        snprintf(nm, 96, "3r3w chunk U%d nt (zero g)", U);
        if (U == 1) rep(nm, 24.0 * n, timeit([&] { k3r3w_chunk<1, true><<<blocks, 256>>>(G4w, M4, V4, n4, 0.9f); }, reps));
        if (U == 2) rep(nm, 24.0 * n, timeit([&] { k3r3w_chunk<2, true><<<blocks, 256>>>(G4w, M4, V4, n4, 0.9f); }, reps));
        if (U == 4) rep(nm, 24.0 * n, timeit([&] { k3r3w_chunk<4, true><<<blocks, 256>>>(G4w, M4, V4, n4, 0.9f); }, reps));
    }
    for (int U : {1, 4, 16}) {
        long blocks = (n4 + 256L * U - 1) / (256L * U);
        char nm[96];
        snprintf(nm, 96, "fill chunk U%d", U);
        if (U == 1) rep(nm, 4.0 * n, timeit([&] { kfill_chunk<1, false><<<blocks, 256>>>(M4, n4); }, reps));
        if (U == 4) rep(nm, 4.0 * n, timeit([&] { kfill_chunk<4, false><<<blocks, 256>>>(M4, n4); }, reps));
        if (U == 16) rep(nm, 4.0 * n, timeit([&] { kfill_chunk<16, false><<<blocks, 256>>>(M4, n4); }, reps));
        snprintf(nm, 96, "fill chunk U%d nt", U);
        if (U == 1) rep(nm, 4.0 * n, timeit([&] { kfill_chunk<1, true><<<blocks, 256>>>(M4, n4); }, reps));
        if (U == 4) rep(nm, 4.0 * n, timeit([&] { kfill_chunk<4, true><<<blocks, 256>>>(M4, n4); }, reps));
        if (U == 16) rep(nm, 4.0 * n, timeit([&] { kfill_chunk<16, true><<<blocks, 256>>>(M4, n4); }, reps));
    }
    for (int grid : {1024, 4096, 16384}) {
        char nm[96];
        snprintf(nm, 96, "fill grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kfill<false><<<grid, 256>>>(M4, n4); }, reps));
        snprintf(nm, 96, "fill nt grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kfill<true><<<grid, 256>>>(M4, n4); }, reps));
    }
    CK(hipMemsetAsync(m, 0, n * 4));
    rep("hipMemsetAsync", 4.0 * n, timeit([&] { CK(hipMemsetAsync(m, 0, n * 4)); }, reps));
    for (int grid : {1024, 2048, 4096, 8192}) {
        if (chunk_only) break;
        char nm[96];
        snprintf(nm, 96, "3r2w U1 grid%d", grid);
        rep(nm, 20.0 * n, timeit([&] { k3r2w<1, false, false><<<grid, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        snprintf(nm, 96, "3r2w U2 grid%d", grid);
        rep(nm, 20.0 * n, timeit([&] { k3r2w<2, false, false><<<grid, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        snprintf(nm, 96, "3r2w U4 grid%d", grid);
        rep(nm, 20.0 * n, timeit([&] { k3r2w<4, false, false><<<grid, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        snprintf(nm, 96, "3r2w U2 ntload+ntstore grid%d", grid);
        rep(nm, 20.0 * n, timeit([&] { k3r2w<2, true, true><<<grid, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        snprintf(nm, 96, "3r2w U2 ntstore grid%d", grid);
        rep(nm, 20.0 * n, timeit([&] { k3r2w<2, false, true><<<grid, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
    }
    for (int U : {1, 2, 4}) {
        long blocks = (n4 + 256L * U - 1) / (256L * U);
        char nm[96];
        snprintf(nm, 96, "3r2w chunk U%d", U);
        if (U == 1) rep(nm, 20.0 * n, timeit([&] { k3r2w_chunk<1, false, false><<<blocks, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        if (U == 2) rep(nm, 20.0 * n, timeit([&] { k3r2w_chunk<2, false, false><<<blocks, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        if (U == 4) rep(nm, 20.0 * n, timeit([&] { k3r2w_chunk<4, false, false><<<blocks, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        snprintf(nm, 96, "3r2w chunk U%d nt", U);
        if (U == 1) rep(nm, 20.0 * n, timeit([&] { k3r2w_chunk<1, true, true><<<blocks, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        if (U == 2) rep(nm, 20.0 * n, timeit([&] { k3r2w_chunk<2, true, true><<<blocks, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
        if (U == 4) rep(nm, 20.0 * n, timeit([&] { k3r2w_chunk<4, true, true><<<blocks, 256>>>(G4, M4, V4, n4, 0.9f); }, reps));
    }
    for (int grid : {2048, 8192}) {
        char nm[96];
        snprintf(nm, 96, "copy grid%d", grid); rep(nm, 8.0 * n, timeit([&] { kcopy<false><<<grid, 256>>>(G4, M4, n4); }, reps));
        snprintf(nm, 96, "copy nt grid%d", grid); rep(nm, 8.0 * n, timeit([&] { kcopy<true><<<grid, 256>>>(G4, M4, n4); }, reps));
        snprintf(nm, 96, "read U1 grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kread<1, false><<<grid, 256>>>(G4, n4, 3.0f, o); }, reps));
        snprintf(nm, 96, "read U4 grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kread<4, false><<<grid, 256>>>(G4, n4, 3.0f, o); }, reps));
        snprintf(nm, 96, "read U8 grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kread<8, false><<<grid, 256>>>(G4, n4, 3.0f, o); }, reps));
        snprintf(nm, 96, "read U4 nt grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kread<4, true><<<grid, 256>>>(G4, n4, 3.0f, o); }, reps));
        snprintf(nm, 96, "fill grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kfill<false><<<grid, 256>>>(M4, n4); }, reps));
        snprintf(nm, 96, "fill nt grid%d", grid); rep(nm, 4.0 * n, timeit([&] { kfill<true><<<grid, 256>>>(M4, n4); }, reps));
    }
    return 0;
}
