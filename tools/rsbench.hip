// K3's one-workgroup radix select (rs_small_wg, the model sets' sampled threshold),
// 54 tensors per launch like ResNet-50's k_rs_small_multi (v0: a previous body kept
// here, v1: the product body). Prints us per launch and checks that the two
// bodies agree on every case (ties, NaN, inf, tiny n, large k).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I adam-compression_amd/csrc -I include
//        tools/rsbench.hip -o tools/rsbench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__device__ unsigned long long g_st[16];
#define RS_STAMP(i) do { __syncthreads(); if (blockIdx.x == 0 && threadIdx.x == 0) g_st[i] = wall_clock64(); } while (0)
#include "radix_select.hpp"
#define RS_STAMP_PREV(i) do { } while (0)
namespace dgc {
__device__ void rs_small_prev(const float* __restrict__ x, int64_t n, uint64_t k64, float* out) {
    constexpr int kPer = kSmallN / kScanThreads;
    __shared__ uint32_t h[kRsBins];
    __shared__ uint32_t lds32[16];
    __shared__ uint32_t nan_cnt, prefix, k_rem, sel_above;
    __shared__ int sel_bin;
    const int tid = threadIdx.x;
    const int nn = (int)n;   // <= kSmallN
    const uint32_t k = (uint32_t)k64;
    RS_STAMP_PREV(0);
    for (int b = tid; b < kRsBins; b += kScanThreads) h[b] = 0;
    if (tid == 0) {
        nan_cnt = 0;
        prefix = 0;
        k_rem = k;
        sel_bin = -1;
    }
    // the thread's keys stay in registers (kPer VGPRs); out-of-range slots hold 0 and
    // are masked by `in` below
    uint32_t key[kPer];
    uint32_t mx = 0, my_nan = 0;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int i = tid + j * kScanThreads;
        key[j] = i < nn ? abs_key(x[i]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const bool in = tid + j * kScanThreads < nn;
        mx = in && key[j] > mx ? key[j] : mx;
        my_nan += in && key[j] > 0x7F800000u ? 1u : 0u;
    }
    __syncthreads();   // h zeroed
    RS_STAMP_PREV(1);
    if (my_nan) atomicAdd(&nan_cnt, my_nan);
    if (tid < nn) atomicAdd(&h[mx >> 21], 1u);
    __syncthreads();
    {
        int bin;
        uint32_t above;
        if (pick_bin_small<2>(h, k, lds32, &bin, &above)) sel_bin = bin;
    }
    __syncthreads();
    const uint32_t floor = sel_bin >= 0 ? (uint32_t)sel_bin << 21 : 0u;
    RS_STAMP_PREV(2);
    for (int pass = 0; pass < 3; ++pass) {
        for (int b = tid; b < kRsBins; b += kScanThreads) h[b] = 0;
        __syncthreads();   // everyone has read sel_bin / prefix
        if (tid == 0) sel_bin = -1;
        const uint32_t pmask = rs_pmask(pass), dmask = rs_dmask(pass), pre = prefix;
        const int shift = rs_shift(pass);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const bool in = tid + j * kScanThreads < nn;
            if (in && (pass == 0 ? key[j] >= floor : (key[j] & pmask) == pre))
                atomicAdd(&h[(key[j] >> shift) & dmask], 1u);
        }
        __syncthreads();
        RS_STAMP_PREV(3 + 2 * pass);
        int bin;
        uint32_t above;
        const bool hit = pass == 2 ? pick_bin_small<1>(h, k_rem, lds32, &bin, &above)
                                   : pick_bin_small<2>(h, k_rem, lds32, &bin, &above);
        if (hit) {
            sel_bin = bin;
            sel_above = above;
        }
        __syncthreads();
        if (tid == 0 && sel_bin >= 0) {
            prefix |= (uint32_t)sel_bin << shift;
            k_rem -= sel_above;
        }
        __syncthreads();
        RS_STAMP_PREV(4 + 2 * pass);
        if (sel_bin < 0) break;   // uniform: k exceeds the key count
    }
    if (tid == 0) *out = (nan_cnt || sel_bin < 0) ? __uint_as_float(0x7FC00000u) : __uint_as_float(prefix);
    __syncthreads();
}

}  // namespace dgc

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using namespace dgc;

__global__ void __launch_bounds__(kScanThreads) k_v0(const float* x, const int64_t* n, const uint64_t* k, float* out,
                                                     int64_t stride) {
    rs_small_prev(x + blockIdx.x * stride, n[blockIdx.x], k[blockIdx.x], out + blockIdx.x);
}
__global__ void __launch_bounds__(kScanThreads) k_v1(const float* x, const int64_t* n, const uint64_t* k, float* out,
                                                     int64_t stride) {
    rs_small_wg(x + blockIdx.x * stride, n[blockIdx.x], k[blockIdx.x], out + blockIdx.x);
}

int main() {
    const int T = 54;
    const int64_t stride = kSmallN;
    std::mt19937_64 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    float *dx, *o0, *o1;
    int64_t* dn;
    uint64_t* dk;
    CK(hipMalloc(&dx, T * stride * 4));
    CK(hipMalloc(&o0, T * 4));
    CK(hipMalloc(&o1, T * 4));
    CK(hipMalloc(&dn, T * 8));
    CK(hipMalloc(&dk, T * 8));
    std::vector<float> hx(T * stride);
    std::vector<int64_t> hn(T);
    std::vector<uint64_t> hk(T);
    void* flush;
    const size_t flush_bytes = 512ull << 20;
    CK(hipMalloc(&flush, flush_bytes));
    // per launch: 512 MB memset first (the keys leave the caches, as K1's samples arrive
    // cold from another XCD), then the kernel alone between two events
    auto run = [&](auto kern, float* o, int reps) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        float tot = 0;
        for (int r = 0; r < reps; ++r) {
            if (getenv("RS_FLUSH")) CK(hipMemsetAsync(flush, r & 0xFF, flush_bytes, 0));
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(kern, dim3(T), dim3(kScanThreads), 0, 0, dx, dn, dk, o, stride);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r > 0) tot += ms;
        }
        return tot * 1000.f / (reps - 1);
    };
    int bad = 0;
    // kind: 0 randn x 1e-3, 1 randn with heavy ties (rounded to 3 bits), 2 all equal,
    // 3 randn + a few NaN / inf, 4 tiny n, 5 large k
    for (int kind = 0; kind < 6; ++kind) {
        for (int t = 0; t < T; ++t) {
            int64_t n = kind == 4 ? 1 + (int64_t)(rng() % 2000) : 20000 + (int64_t)(rng() % 12768);
            uint64_t k = kind == 5 ? 1 + rng() % n : (uint64_t)std::ceil(n * 1e-3);
            if (k > (uint64_t)n) k = n;
            hn[t] = n;
            hk[t] = k;
            for (int64_t i = 0; i < n; ++i) {
                float v = nd(rng) * 1e-3f;
                if (kind == 1) v = std::ldexp(std::round(std::ldexp(v, 13)), -13);
                if (kind == 2) v = 0.25f;
                if (kind == 3 && rng() % 5000 == 0) v = (rng() & 1) ? NAN : -INFINITY;
                hx[t * stride + i] = v;
            }
        }
        CK(hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dn, hn.data(), T * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dk, hk.data(), T * 8, hipMemcpyHostToDevice));
        const float t0 = run(k_v0, o0, 50), t1 = run(k_v1, o1, 50);
        std::vector<float> r0(T), r1(T);
        CK(hipMemcpy(r0.data(), o0, T * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r1.data(), o1, T * 4, hipMemcpyDeviceToHost));
        int mism = 0;
        for (int t = 0; t < T; ++t) {
            // reference on the host: k-th largest |x|, NaN if any NaN
            std::vector<uint32_t> keys(hn[t]);
            bool nan = false;
            for (int64_t i = 0; i < hn[t]; ++i) {
                uint32_t b;
                std::memcpy(&b, &hx[t * stride + i], 4);
                keys[i] = b & 0x7FFFFFFFu;
                nan |= keys[i] > 0x7F800000u;
            }
            std::nth_element(keys.begin(), keys.begin() + (hk[t] - 1), keys.end(), std::greater<uint32_t>());
            uint32_t want = nan ? 0x7FC00000u : keys[hk[t] - 1];
            uint32_t g0, g1;
            std::memcpy(&g0, &r0[t], 4);
            std::memcpy(&g1, &r1[t], 4);
            if (g0 != want || g1 != want) ++mism;
        }
        bad += mism;
        printf("kind %d: v0 %.2f us  v1 %.2f us  mismatches %d\n", kind, t0, t1, mism);
        unsigned long long st[16];
        CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_st), sizeof(st)));
        printf("  v1 phases (us from start, block 0):");
        for (int i = 1; i < 9; ++i) printf(" %.2f", (st[i] - st[0]) * 0.01);
        printf("\n");
    }
    printf(bad ? "FAIL\n" : "OK\n");
    return bad ? 1 : 0;
}
