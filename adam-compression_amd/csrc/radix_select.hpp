// K3: k-th largest |x| by MSB-first radix select on the fp32 bit pattern.
//
// Replaces torch.min(torch.topk(samples, k, sorted=False)[0]) (dgc/compression.py:123)
// and, over the candidate set, the resample topk (dgc/compression.py:134-137).
//
// Keys are |x| bit patterns (sign cleared): for non-negative floats uint order is
// float order, +0 == -0, and NaN keys (> 0x7F800000) sort above +inf exactly as
// topk ranks NaN. torch.min over a top-k set that holds a NaN returns NaN, so the
// result is NaN whenever any NaN key exists (counted in pass 0).
//
// Digits: 11 + 11 + 10 bits (2048/2048/1024 bins). Each pass = one histogram
// launch (LDS histogram per block, non-zero bins flushed with 64-bit global
// atomics) + one single-block scan launch that picks the bin holding the k-th
// largest key and narrows (prefix, k). Inputs of <= kSmallN keys run the three
// passes inside ONE workgroup from LDS.
//
// The scalar result is written to a device float; nothing returns to the host.
#pragma once

#include "dgc_common.hpp"

namespace dgc {

constexpr int kRsBins = 2048;
constexpr int kSmallN = 32768;
constexpr int kScanThreads = 1024;

struct RSState {
    uint32_t prefix;
    uint32_t found;
    uint64_t k_rem;
    uint64_t nan_count;
    uint64_t pad;
    unsigned long long hist[kRsBins];
};

__host__ __device__ constexpr int rs_shift(int pass) { return pass == 0 ? 21 : pass == 1 ? 10 : 0; }
__host__ __device__ constexpr uint32_t rs_dmask(int pass) { return pass == 2 ? 0x3FFu : 0x7FFu; }
__host__ __device__ constexpr uint32_t rs_pmask(int pass) {
    return pass == 0 ? 0u : pass == 1 ? 0xFFE00000u : 0xFFFFFC00u;
}
__host__ __device__ constexpr int rs_bins(int pass) { return pass == 2 ? 1024 : 2048; }

// ---------------------------------------------------------------- key sources
// Dense array of floats (the strided samples, or a full tensor).
struct DenseKeys {
    const float* x;
    int64_t n;
    template <class F>
    __device__ __forceinline__ void visit(F&& f) const {
        const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        const int64_t G = (int64_t)gridDim.x * blockDim.x;
        if (aligned16(x)) {
            const int64_t n4 = n / 4;
            const float4* x4 = reinterpret_cast<const float4*>(x);
            for (int64_t i = tid; i < n4; i += G) {
                const float4 v = x4[i];
                f(abs_key(v.x));
                f(abs_key(v.y));
                f(abs_key(v.z));
                f(abs_key(v.w));
            }
            for (int64_t i = n4 * 4 + tid; i < n; i += G) f(abs_key(x[i]));
        } else {
            for (int64_t i = tid; i < n; i += G) f(abs_key(x[i]));
        }
    }
};

// ---------------------------------------------------------------- block scan
// Exclusive scan of one u64 per thread over a 1024-thread block; returns the
// exclusive prefix and writes the block total to *total (all threads).
__device__ __forceinline__ uint64_t block_exclusive_scan_1024(uint64_t v, uint64_t* lds16,
                                                              uint64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) lds16[wid] = incl;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        const uint64_t s = lds16[w];
        if (w < wid) wbase += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + incl - v;
}

// Pick the bin of the k-th largest key from counts[0..bins) (one block of 1024).
// Thread t owns descending positions {2t, 2t+1} (2048 bins) or {t} (1024 bins).
// Returns true in exactly one thread, setting *bin and *above (keys in higher bins).
template <typename CountT>
__device__ __forceinline__ bool pick_bin(const CountT* counts, int bins, uint64_t k,
                                         uint64_t* lds16, int* bin, uint64_t* above) {
    const int per = bins / kScanThreads;   // 2 or 1
    const int t = threadIdx.x;
    uint64_t c[2] = {0, 0};
    for (int j = 0; j < per; ++j) c[j] = counts[bins - 1 - (per * t + j)];
    uint64_t total;
    uint64_t run = block_exclusive_scan_1024(c[0] + c[1], lds16, &total);
    bool hit = false;
    for (int j = 0; j < per; ++j) {
        if (!hit && run < k && k <= run + c[j]) {
            hit = true;
            *bin = bins - 1 - (per * t + j);
            *above = run;
        }
        run += c[j];
    }
    return hit;
}

// ---------------------------------------------------------------- kernels
template <class Src>
__global__ void __launch_bounds__(kBlock)
k_rs_hist(Src src, RSState* st, int pass, const int32_t* gate) {
    if (gate && *gate == 0) return;
    __shared__ uint32_t h[kRsBins];
    __shared__ uint32_t nan_cnt;
    for (int b = threadIdx.x; b < kRsBins; b += kBlock) h[b] = 0;
    if (threadIdx.x == 0) nan_cnt = 0;
    __syncthreads();
    const uint32_t prefix = st->prefix;
    const uint32_t pmask = rs_pmask(pass), dmask = rs_dmask(pass);
    const int shift = rs_shift(pass);
    src.visit([&](uint32_t key) {
        if ((key & pmask) == prefix) atomicAdd(&h[(key >> shift) & dmask], 1u);
        if (pass == 0 && key > 0x7F800000u) atomicAdd(&nan_cnt, 1u);
    });
    __syncthreads();
    for (int b = threadIdx.x; b < rs_bins(pass); b += kBlock)
        if (h[b]) atomicAdd(&st->hist[b], (unsigned long long)h[b]);
    if (pass == 0 && threadIdx.x == 0 && nan_cnt)
        atomicAdd((unsigned long long*)&st->nan_count, (unsigned long long)nan_cnt);
}

__global__ void __launch_bounds__(kScanThreads)
k_rs_scan(RSState* st, int pass, float* out, const int32_t* gate) {
    if (gate && *gate == 0) return;
    __shared__ uint64_t lds16[16];
    __shared__ int sel_bin;
    __shared__ uint64_t sel_above;
    if (threadIdx.x == 0) sel_bin = -1;
    __syncthreads();
    const uint64_t k = st->k_rem;
    int bin;
    uint64_t above;
    if (pick_bin(st->hist, rs_bins(pass), k, lds16, &bin, &above)) {
        sel_bin = bin;
        sel_above = above;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kRsBins; b += kScanThreads) st->hist[b] = 0;
    if (threadIdx.x == 0) {
        if (sel_bin < 0) {
            st->found = 0;   // k exceeded the key count: report NaN
            if (out) *out = __uint_as_float(0x7FC00000u);
        } else {
            st->prefix |= (uint32_t)sel_bin << rs_shift(pass);
            st->k_rem = k - sel_above;
            if (pass == 2) {
                st->found = 1;
                if (out) *out = st->nan_count ? __uint_as_float(0x7FC00000u) : __uint_as_float(st->prefix);
            }
        }
    }
}

__global__ void k_rs_init(RSState* st, uint64_t k, const int32_t* gate) {
    if (gate && *gate == 0) return;
    for (int b = threadIdx.x; b < kRsBins; b += blockDim.x) st->hist[b] = 0;
    if (threadIdx.x == 0) {
        st->prefix = 0;
        st->found = 0;
        st->k_rem = k;
        st->nan_count = 0;
    }
}

// All three passes in one 1024-thread workgroup, keys staged in LDS.
__global__ void __launch_bounds__(kScanThreads)
k_rs_small(const float* __restrict__ x, int64_t n, uint64_t k, float* out) {
    __shared__ uint32_t keys[kSmallN];
    __shared__ uint32_t h[kRsBins];
    __shared__ uint64_t lds16[16];
    __shared__ uint32_t nan_cnt, prefix;
    __shared__ uint64_t k_rem;
    __shared__ int sel_bin;
    __shared__ uint64_t sel_above;
    if (threadIdx.x == 0) {
        nan_cnt = 0;
        prefix = 0;
        k_rem = k;
    }
    __syncthreads();
    uint32_t my_nan = 0;
    for (int i = threadIdx.x; i < n; i += kScanThreads) {
        const uint32_t key = abs_key(x[i]);
        keys[i] = key;
        my_nan += key > 0x7F800000u;
    }
    if (my_nan) atomicAdd(&nan_cnt, my_nan);
    for (int pass = 0; pass < 3; ++pass) {
        for (int b = threadIdx.x; b < kRsBins; b += kScanThreads) h[b] = 0;
        if (threadIdx.x == 0) sel_bin = -1;
        __syncthreads();
        const uint32_t pmask = rs_pmask(pass), dmask = rs_dmask(pass), pre = prefix;
        const int shift = rs_shift(pass);
        for (int i = threadIdx.x; i < n; i += kScanThreads) {
            const uint32_t key = keys[i];
            if ((key & pmask) == pre) atomicAdd(&h[(key >> shift) & dmask], 1u);
        }
        __syncthreads();
        int bin;
        uint64_t above;
        if (pick_bin(h, rs_bins(pass), k_rem, lds16, &bin, &above)) {
            sel_bin = bin;
            sel_above = above;
        }
        __syncthreads();
        if (threadIdx.x == 0 && sel_bin >= 0) {
            prefix |= (uint32_t)sel_bin << shift;
            k_rem -= sel_above;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        *out = (nan_cnt || sel_bin < 0) ? __uint_as_float(0x7FC00000u) : __uint_as_float(prefix);
}

// Host launcher over any key source. `gate` (device int, may be null) turns every
// launch into a no-op when zero, so the chain can sit in a device-decided pipeline.
template <class Src>
inline int radix_select_launch(const Src& src, int64_t work_items, uint64_t k, float* out,
                               RSState* st, const int32_t* gate, hipStream_t s) {
    hipLaunchKernelGGL(k_rs_init, dim3(1), dim3(kBlock), 0, s, st, k, gate);
    DGC_LAUNCHED();
    const int grid = grid_for(work_items, kBlock * 4);
    for (int pass = 0; pass < 3; ++pass) {
        hipLaunchKernelGGL((k_rs_hist<Src>), dim3(grid), dim3(kBlock), 0, s, src, st, pass, gate);
        DGC_LAUNCHED();
        hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(kScanThreads), 0, s, st, pass, out, gate);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

}  // namespace dgc
