// K3: k-th largest |x| by MSB-first radix select on the fp32 bit pattern, for one
// or many independent key sets in the same launches.
//
// Replaces torch.min(torch.topk(samples, k, sorted=False)[0]) (dgc/compression.py:123)
// per compressed tensor and, over the candidate set, the value of the resample topk's
// k-th key on its partial_sort path (dgc/compression.py:134-137).
//
// Keys are |x| bit patterns (sign cleared): for non-negative floats uint order is
// float order, +0 == -0, and NaN keys (> 0x7F800000) sort above +inf exactly as
// topk ranks NaN. torch.min over a top-k set that holds a NaN returns NaN, so the
// result is NaN whenever any NaN key exists (counted in pass 0).
//
// Digits: 11 + 11 + 10 bits (2048/2048/1024 bins). One launch per pass covers every
// key set ("task"): each workgroup serves ONE task (a prefix table of block counts
// maps blockIdx to the task), builds an LDS histogram of the task's keys that match
// the task's current prefix and flushes its non-zero bins with 64-bit device atomics
// into the task's state; the LAST of the task's workgroups to arrive (agent-scope
// atomics both sides, cdna_hip_programming.md G16) picks the bin holding the k-th
// largest key and narrows (prefix, k) for the next pass. Tasks of <= kSmallN keys run
// all three passes inside ONE workgroup from LDS (k_rs_small, one workgroup per task).
//
// Results are device floats; nothing returns to the host.
#pragma once

#include "dgc_common.hpp"

namespace dgc {

constexpr int kRsBins = 2048;

#ifdef DGC_K5_PROF
// tools/k3_prof.py (profiling build, make k5prof): per-workgroup wall-clock stamps of the
// one-workgroup thresholds (k_rs_small_multi, workgroup = task < 64) — 0 start, 1 keys
// loaded + pass-0 floor, 2 floor picked, 3..8 each pass's histogram / pick, 9 threshold
// written, 10 selection state reset, 11 kernel end
__device__ unsigned long long g_rs_prof[64][12];
#define RS_STAMP(i) \
    do { if (threadIdx.x == 0 && blockIdx.x < 64) g_rs_prof[blockIdx.x][i] = wall_clock64(); } while (0)
#else
#define RS_STAMP(i) do { } while (0)
#endif
constexpr int kSmallN = 32768;
constexpr int kScanThreads = 1024;

struct RSState {
    uint32_t prefix;
    uint32_t found;
    uint64_t k_rem;
    uint64_t nan_count;
    uint32_t tickets[4];
    uint32_t win_n;                    // > 0: the passes read the K1 sample window list of
                                       // win_n keys instead of the samples (select.hip)
    uint32_t small_done;               // select.hip: a window of <= kSmallN keys was selected
                                       // in one workgroup; the passes skip the task
    unsigned long long hist[3][kRsBins];
};

__host__ __device__ constexpr int rs_shift(int pass) { return pass == 0 ? 21 : pass == 1 ? 10 : 0; }
__host__ __device__ constexpr uint32_t rs_dmask(int pass) { return pass == 2 ? 0x3FFu : 0x7FFu; }
__host__ __device__ constexpr uint32_t rs_pmask(int pass) {
    return pass == 0 ? 0u : pass == 1 ? 0xFFE00000u : 0xFFFFFC00u;
}
__host__ __device__ constexpr int rs_bins(int pass) { return pass == 2 ? 1024 : 2048; }

// The task served by block b, from an ascending prefix table blk[0..T] of block counts
// (blk[T] = grid, blk[0] = 0): the largest t with blk[t] <= b = (#entries <= b) - 1.
// Each wave counts 64 entries per load with a ballot — one round trip for T <= 64
// where a binary search is log2(T) dependent ones, paid at the start of every block
// of every batched launch. Call from whole waves; every lane gets the same t.
__device__ __forceinline__ int task_of_block(const int32_t* blk, int T, int b) {
    if (T <= 1) return 0;
    const int lane = threadIdx.x & 63;
    int cnt = 0;
    for (int i0 = 0; i0 < T; i0 += 64) {
        const int i = i0 + lane;
        const uint64_t m = __ballot(i < T && blk[i] <= b);
        cnt += __popcll(m);
        if (m != ~0ull) break;   // ascending table: every later entry is > b
    }
    return __builtin_amdgcn_readfirstlane(cnt - 1);
}

// Strided visit of n floats' keys by the `nb` blocks of one task (lb = block index in the task).
template <class F>
__device__ __forceinline__ void visit_dense(const float* x, int64_t n, int64_t lb, int64_t nb, F&& f) {
    const int64_t tid = lb * blockDim.x + threadIdx.x;
    const int64_t G = nb * blockDim.x;
    if (aligned16(x)) {
        // kVisitBatch float4 loads in flight per lane before any key is used: the
        // histogram's LDS atomics would otherwise serialise one load round trip each
        constexpr int kVisitBatch = 8;
        const int64_t n4 = n / 4;
        const float4* x4 = reinterpret_cast<const float4*>(x);
        for (int64_t i0 = tid; i0 < n4; i0 += kVisitBatch * G) {
            float4 v[kVisitBatch];
#pragma unroll
            for (int u = 0; u < kVisitBatch; ++u)
                if (i0 + u * G < n4) v[u] = x4[i0 + u * G];
#pragma unroll
            for (int u = 0; u < kVisitBatch; ++u)
                if (i0 + u * G < n4) {
                    f(abs_key(v[u].x));
                    f(abs_key(v[u].y));
                    f(abs_key(v[u].z));
                    f(abs_key(v[u].w));
                }
        }
        for (int64_t i = n4 * 4 + tid; i < n; i += G) f(abs_key(x[i]));
    } else {
        for (int64_t i = tid; i < n; i += G) f(abs_key(x[i]));
    }
}

// One dense key set: dgc_kth_largest.
struct DenseKeys {
    const float* x;
    int64_t n;
    RSState* st;
    float* result;
    __device__ __forceinline__ int task(int) const { return 0; }
    __device__ __forceinline__ int first_block(int) const { return 0; }
    __device__ __forceinline__ int blocks(int) const { return (int)gridDim.x; }
    __device__ __forceinline__ bool active(int) const { return true; }
    __device__ __forceinline__ RSState* state(int) const { return st; }
    __device__ __forceinline__ float* out(int) const { return result; }
    __device__ __forceinline__ void done(int) const {}
    template <class F>
    __device__ __forceinline__ void visit(int, int64_t lb, int64_t nb, F&& f) const {
        visit_dense(x, n, lb, nb, f);
    }
};

template <typename CountT>
__device__ __forceinline__ uint64_t load_count(const CountT* p) {
    return (uint64_t)*p;
}
// totals flushed by other workgroups' atomics: read them where atomics are performed
__device__ __forceinline__ uint64_t load_count(const unsigned long long* p) {
    return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Pick the bin of the k-th largest key from counts[0..bins). Thread t owns the
// descending positions [per*t, per*t + per), per <= kPickMax. Returns true in exactly
// one thread. The thread's counts are loaded once, all in flight together (unrolled,
// predicated): a loop of dependent agent-scope loads costs a full L2 round trip per
// bin, ~1 us each, and the last workgroup of every radix pass runs this.
constexpr int kPickMax = 16;
template <typename CountT>
__device__ __forceinline__ bool pick_bin(const CountT* counts, int bins, uint64_t k, uint64_t* lds16, int* bin,
                                         uint64_t* above) {
    const int per = bins / (int)blockDim.x;
    const int t = threadIdx.x;
    uint64_t c[kPickMax];
#pragma unroll
    for (int j = 0; j < kPickMax; ++j) c[j] = j < per ? load_count(&counts[bins - 1 - (per * t + j)]) : 0;
    uint64_t sum = 0;
#pragma unroll
    for (int j = 0; j < kPickMax; ++j) sum += c[j];
    uint64_t total;
    uint64_t run = block_exclusive_scan(sum, lds16, &total);
    bool hit = false;
    if (run < k && k <= run + sum) {
#pragma unroll
        for (int j = 0; j < kPickMax; ++j) {
            if (!hit && j < per && run < k && k <= run + c[j]) {
                hit = true;
                *bin = bins - 1 - (per * t + j);
                *above = run;
            }
            run += c[j];
        }
    }
    return hit;
}

// ---------------------------------------------------------------- kernels
__device__ __forceinline__ void rs_reset(RSState* st, uint64_t k) {
    for (int b = threadIdx.x; b < 3 * kRsBins; b += blockDim.x) (&st->hist[0][0])[b] = 0;
    if (threadIdx.x == 0) {
        st->prefix = 0;
        st->found = 0;
        st->k_rem = k;
        st->nan_count = 0;
        for (int i = 0; i < 4; ++i) st->tickets[i] = 0;
        st->win_n = 0;
    }
}

__global__ void k_rs_init(RSState* st, uint64_t k) { rs_reset(st, k); }

template <class Src>
__device__ __forceinline__ void rs_hist_body(const Src& src, int pass, int bx) {
    const int t = src.task(bx);
    if (!src.active(t)) return;   // uniform per workgroup
    if (bx - src.first_block(t) >= src.blocks(t)) return;   // not a participant of the task
    __shared__ uint32_t h[kRsBins];
    __shared__ uint32_t nan_cnt;
    __shared__ uint64_t lds16[16];
    __shared__ int sel_bin;
    __shared__ uint64_t sel_above;
    RSState* st = src.state(t);
    for (int b = threadIdx.x; b < kRsBins; b += kBlock) h[b] = 0;
    if (threadIdx.x == 0) {
        nan_cnt = 0;
        sel_bin = -1;
    }
    __syncthreads();
    const uint32_t prefix = st->prefix;
    const uint32_t pmask = rs_pmask(pass), dmask = rs_dmask(pass);
    const int shift = rs_shift(pass);
    const int b0 = src.first_block(t), nb = src.blocks(t);
    src.visit(t, (int64_t)bx - b0, nb, [&](uint32_t key) {
        if ((key & pmask) == prefix) atomicAdd(&h[(key >> shift) & dmask], 1u);
        if (pass == 0 && key > 0x7F800000u) atomicAdd(&nan_cnt, 1u);
    });
    __syncthreads();
    unsigned long long* gh = st->hist[pass];
    for (int b = threadIdx.x; b < rs_bins(pass); b += kBlock)
        if (h[b]) atomicAdd(&gh[b], (unsigned long long)h[b]);
    if (pass == 0 && threadIdx.x == 0 && nan_cnt)
        atomicAdd((unsigned long long*)&st->nan_count, (unsigned long long)nan_cnt);
    if (!last_block_arrival(&st->tickets[pass], (uint32_t)nb)) return;
    // the last workgroup of the task picks the bin for the task
    const uint64_t k = st->k_rem;
    int bin;
    uint64_t above;
    if (pick_bin(gh, rs_bins(pass), k, lds16, &bin, &above)) {
        sel_bin = bin;
        sel_above = above;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float* out = src.out(t);
        if (sel_bin < 0) {
            st->found = 0;   // k exceeded the key count: report NaN
            if (out) *out = __uint_as_float(0x7FC00000u);
        } else {
            st->prefix = prefix | ((uint32_t)sel_bin << shift);
            st->k_rem = k - sel_above;
            if (pass == 2) {
                st->found = 1;
                const uint64_t nans = __hip_atomic_load((unsigned long long*)&st->nan_count, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
                if (out) *out = nans ? __uint_as_float(0x7FC00000u) : __uint_as_float(st->prefix);
            }
        }
    }
    if (pass == 2) {   // the task's k-th largest key is known: the source's follow-up
        __syncthreads();
        src.done(t);
    }
}

// Exclusive scan of one u32 per thread over a kScanThreads workgroup (lds32: 16
// words); returns the prefix, *total the workgroup total. Two barriers.
__device__ __forceinline__ uint32_t block_exclusive_scan32(uint32_t v, uint32_t* lds32, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan<DppAdd>(v);
    if (lane == 63) lds32[wid] = incl;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
        const uint32_t s = lds32[w];
        wbase += w < wid ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + incl - v;
}

// pick_bin for u32 LDS counts of PER bins per thread (bins = PER * kScanThreads): true
// in the one thread whose bins hold the k-th largest key; *bin, *above as pick_bin.
template <int PER>
__device__ __forceinline__ bool pick_bin_small(const uint32_t* h, uint32_t k, uint32_t* lds32, int* bin,
                                               uint32_t* above) {
    constexpr int bins = PER * kScanThreads;
    const int t = threadIdx.x;
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        c[j] = h[bins - 1 - (PER * t + j)];
        sum += c[j];
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan32(sum, lds32, &total);
    bool hit = false;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        if (!hit && run < k && k <= run + c[j]) {
            hit = true;
            *bin = bins - 1 - (PER * t + j);
            *above = run;
        }
        run += c[j];
    }
    return hit;
}

// Keys of x[0, nn) (nn >= 4, x 16-B aligned) into registers, PER per thread: element
// 4 * (tid + j4 * kScanThreads) + e -> key[4 * j4 + e], 0 past nn. Every 16-B load is
// issued, in bounds (a float4 past the whole ones re-reads the last whole one), before
// any is used: a load under an if / else per float4 made the compiler wait out each one
// before the next (8 round trips, ~8 us of K3 at 32k samples); the partial float4
// (nn & 3 elements) is read after, by the thread that owns it.
template <int PER>
__device__ __forceinline__ void load_keys4(const float* __restrict__ x, int nn, uint32_t (&key)[PER]) {
    const int tid = threadIdx.x;
    const int nf4 = nn >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    float4 f[PER / 4];
#pragma unroll
    for (int j4 = 0; j4 < PER / 4; ++j4) {
        const int q = tid + j4 * kScanThreads;
        f[j4] = x4[q < nf4 ? q : nf4 - 1];
    }
#pragma unroll
    for (int j4 = 0; j4 < PER / 4; ++j4) {
        const bool in = tid + j4 * kScanThreads < nf4;
        key[4 * j4] = in ? abs_key(f[j4].x) : 0u;
        key[4 * j4 + 1] = in ? abs_key(f[j4].y) : 0u;
        key[4 * j4 + 2] = in ? abs_key(f[j4].z) : 0u;
        key[4 * j4 + 3] = in ? abs_key(f[j4].w) : 0u;
    }
    if ((nn & 3) && nf4 % kScanThreads == tid) {
#pragma unroll
        for (int j4 = 0; j4 < PER / 4; ++j4)
            if (j4 == nf4 / kScanThreads)
#pragma unroll
                for (int e = 0; e < 3; ++e)
                    if (e < (nn & 3)) key[4 * j4 + e] = abs_key(x[4 * nf4 + e]);
    }
}

// All three passes of one key set of <= kSmallN keys in ONE 1024-thread workgroup
// (k_rs_small, k_rs_small_multi): x[0..n) -> *out = k-th largest |x| (NaN if any |x|
// is NaN). Every key load in flight at once (kSmallN / kScanThreads per
// thread) into LDS, u32 counts and scans, and pass 0 floored. Pass 0's LDS histogram
// atomics all land in the few bins the keys' exponents span (~n serialised
// same-address adds), so it first histograms the per-thread maxima (<= 1024 adds) and
// picks the bin b0 holding their k-th largest: at least k distinct keys (those maxima)
// are >= b0 << 21, so the k-th largest key is too, and pass 0 need count only the keys
// >= b0 << 21 — the bins >= b0 are exact, pick_bin picks the same bin. No floor when
// fewer than k threads hold a key.
__device__ __forceinline__ void rs_small_wg(const float* __restrict__ x, int64_t n, uint64_t k64, float* out) {
    constexpr int kPer = kSmallN / kScanThreads;
    __shared__ uint32_t h[kRsBins];
    __shared__ uint32_t lds32[16];
    __shared__ uint32_t nan_cnt, prefix, k_rem, sel_above;
    __shared__ int sel_bin;
    const int tid = threadIdx.x;
    const int nn = (int)n;   // <= kSmallN
    const uint32_t k = (uint32_t)k64;
    RS_STAMP(0);
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
    if (aligned16(x) && nn >= 4) {
        load_keys4<kPer>(x, nn, key);
    } else {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const int i = tid + j * kScanThreads;
            key[j] = i < nn ? abs_key(x[i]) : 0u;
        }
    }
    // element index of key[j] (the two layouts above)
    auto elem = [&](int j) -> int {
        return aligned16(x) && nn >= 4 ? 4 * (tid + (j / 4) * kScanThreads) + (j & 3) : tid + j * kScanThreads;
    };
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const bool in = elem(j) < nn;
        mx = in && key[j] > mx ? key[j] : mx;
        my_nan += in && key[j] > 0x7F800000u ? 1u : 0u;
    }
    __syncthreads();   // h zeroed
    RS_STAMP(1);
    if (my_nan) atomicAdd(&nan_cnt, my_nan);
    if (elem(0) < nn) atomicAdd(&h[mx >> 21], 1u);   // the thread holds a key
    __syncthreads();
    {
        int bin;
        uint32_t above;
        if (pick_bin_small<2>(h, k, lds32, &bin, &above)) sel_bin = bin;
    }
    __syncthreads();
    const uint32_t floor = sel_bin >= 0 ? (uint32_t)sel_bin << 21 : 0u;
    RS_STAMP(2);
    for (int pass = 0; pass < 3; ++pass) {
        for (int b = tid; b < kRsBins; b += kScanThreads) h[b] = 0;
        __syncthreads();   // everyone has read sel_bin / prefix
        if (tid == 0) sel_bin = -1;
        const uint32_t pmask = rs_pmask(pass), dmask = rs_dmask(pass), pre = prefix;
        const int shift = rs_shift(pass);
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const bool in = elem(j) < nn;
            if (in && (pass == 0 ? key[j] >= floor : (key[j] & pmask) == pre))
                atomicAdd(&h[(key[j] >> shift) & dmask], 1u);
        }
        __syncthreads();
        RS_STAMP(3 + 2 * pass);
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
        RS_STAMP(4 + 2 * pass);
        if (sel_bin < 0) break;   // uniform: k exceeds the key count
    }
    if (tid == 0) *out = (nan_cnt || sel_bin < 0) ? __uint_as_float(0x7FC00000u) : __uint_as_float(prefix);
    __syncthreads();
    RS_STAMP(9);
}

// The k-th largest |x| of a K1 sample WINDOW (select.hip: every sample with key >= the
// window threshold, ks..kWinMax of them) in ONE 1024-thread workgroup, PER keys per
// thread in registers. The window's keys all sit within a few octaves above its
// threshold — the few bins of their exponents, where a fixed-digit pass 0 serialises
// ~n LDS atomics on a handful of addresses (76 us at 83k keys) and the maxima floor of
// rs_small_wg does not apply (k above the thread count) — so the digits are taken from
// key - min instead, 12 bits at a time from the top of the span (4096 bins: two passes
// for a span below 2^24 key units), as the resample set path does. NaN anywhere: NaN.
constexpr int kWinPer = 64;
constexpr int kWinMax = kWinPer * kScanThreads;   // 65536 keys
__device__ __forceinline__ void rs_window_wg(const float* __restrict__ x, int64_t n, uint64_t k64, float* out) {
    constexpr int kBins = 4096;
    __shared__ uint32_t h[kBins];
    __shared__ uint32_t lds32[16];
    __shared__ uint32_t red[3][kScanThreads / kWave];
    __shared__ uint32_t sel_above;
    __shared__ int sel_bin;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int nn = (int)n;   // <= kWinMax
    const uint32_t k = (uint32_t)k64;
    // element 4 * (tid + j4 * 1024) + e -> key[4 * j4 + e] (16-B loads; the window is 16-B aligned)
    uint32_t key[kWinPer];
    if (nn >= 4) {
        load_keys4<kWinPer>(x, nn, key);
    } else {
#pragma unroll
        for (int j = 0; j < kWinPer; ++j) key[j] = (j & ~3) == 0 && tid == 0 && j < nn ? abs_key(x[j]) : 0u;
    }
    auto in = [&](int j) { return 4 * (tid + (j / 4) * kScanThreads) + (j & 3) < nn; };
    uint32_t mn = 0xFFFFFFFFu, mx = 0, nan = 0;
#pragma unroll
    for (int j = 0; j < kWinPer; ++j)
        if (in(j)) {
            nan |= key[j] > 0x7F800000u ? 1u : 0u;
            mn = key[j] < mn ? key[j] : mn;
            mx = key[j] > mx ? key[j] : mx;
        }
    mn = wave_min_u32(mn);
    mx = wave_max(mx);
    nan = wave_max(nan);
    if (lane == 0) {
        red[0][wv] = mn;
        red[1][wv] = mx;
        red[2][wv] = nan;
    }
    for (int b = tid; b < kBins; b += kScanThreads) h[b] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kScanThreads / kWave; ++i) {
        mn = red[0][i] < mn ? red[0][i] : mn;
        mx = red[1][i] > mx ? red[1][i] : mx;
        nan |= red[2][i];
    }
    if (nan || k == 0 || k > (uint32_t)nn) {   // uniform
        if (tid == 0) *out = __uint_as_float(0x7FC00000u);
        __syncthreads();
        return;
    }
    const uint32_t span = mx - mn;
    int hi = span ? 32 - __builtin_clz(span) : 0;
    uint32_t prefix = 0, k_rem = k;
    while (hi > 0) {
        const int lo = hi > 12 ? hi - 12 : 0;
#pragma unroll
        for (int j = 0; j < kWinPer; ++j) {
            const uint32_t v = key[j] - mn;
            if (in(j) && (hi >= 32 || (v >> hi) == prefix)) atomicAdd(&h[(v >> lo) & ((1u << (hi - lo)) - 1u)], 1u);
        }
        if (tid == 0) sel_bin = -1;
        __syncthreads();
        int bin;
        uint32_t above;
        if (pick_bin_small<4>(h, k_rem, lds32, &bin, &above)) {
            sel_bin = bin;
            sel_above = above;
        }
        __syncthreads();
        const int sb = sel_bin;
        const uint32_t a = sel_above;
        __syncthreads();   // every thread has read sel_*
        for (int b = tid; b < kBins; b += kScanThreads) h[b] = 0;
        __syncthreads();   // zeroed before the next pass's adds (a wave ahead lost counts to a late zero)
        if (sb < 0) {   // (cannot happen: k <= n)
            if (tid == 0) *out = __uint_as_float(0x7FC00000u);
            __syncthreads();
            return;
        }
        prefix = (prefix << (hi - lo)) | (uint32_t)sb;
        k_rem -= a;
        hi = lo;
    }
    if (tid == 0) *out = __uint_as_float(mn + prefix);
    __syncthreads();
}

// K1 also histograms the window as it appends to it (select.hip k_compensate_list): one
// agent atomic per windowed sample (~3 ks of the S samples) into kWinBins bins of
// 2^kWinShift key units above the window key — bins 0 .. kWinBins - 3 span a factor
// of ~1.4 in |x| —, the keys past that range in bin kWinBins - 2 and NaN in the last.
constexpr int kWinBins = 4096;
constexpr int kWinShift = 10;
constexpr int kWinBinCap = 4096;   // keys of the k-th key's bin gathered on chip
__device__ __forceinline__ uint32_t win_bin(uint32_t key, uint32_t wk) {
    if (key > 0x7F800000u) return kWinBins - 1;   // NaN
    const uint32_t b = (key - wk) >> kWinShift;   // key >= wk: a windowed sample
    return b < (uint32_t)(kWinBins - 2) ? b : (uint32_t)(kWinBins - 2);
}

// The k-th largest key of a COMPLETE window (all cnt of its keys in x) from K1's
// histogram gh, in one workgroup, re-zeroing gh for the next call: the bin of the k-th
// key from a scan of the 4096 counts (no pass over the keys), then that bin's keys —
// one read of the window, ~100 of them at 1B — in one exact 1024-bin pass over their
// low kWinShift bits. Returns false, *out untouched, when the k-th key lies past the
// binned range or its bin holds more than kWinBinCap keys (rs_window_wg or the passes
// then take the window); NaN in the window: NaN, as rs_window_wg.
__device__ __forceinline__ bool rs_window_hist_wg(const float* __restrict__ x, uint32_t cnt,
                                                  uint32_t* __restrict__ gh, uint32_t wk, uint32_t k,
                                                  float* out) {
    __shared__ uint32_t h[kWinBins];
    __shared__ uint32_t buf[kWinBinCap];
    __shared__ uint32_t lds32[16];
    __shared__ uint32_t sel_above, nbuf;
    __shared__ int sel_bin;
    const int tid = threadIdx.x, lane = tid & 63;
    for (int q = tid; q < kWinBins; q += kScanThreads) {
        h[q] = gh[q];
        gh[q] = 0;
    }
    if (tid == 0) {
        sel_bin = -1;
        nbuf = 0;
    }
    __syncthreads();
    if (h[kWinBins - 1]) {   // uniform: a NaN sample
        if (tid == 0) *out = __uint_as_float(0x7FC00000u);
        __syncthreads();
        return true;
    }
    int bin;
    uint32_t above;
    if (pick_bin_small<kWinBins / kScanThreads>(h, k, lds32, &bin, &above)) {
        sel_bin = bin;
        sel_above = above;
    }
    __syncthreads();
    const int b = sel_bin;
    const uint32_t a = sel_above;
    if (b < 0 || b >= kWinBins - 2 || h[b] > (uint32_t)kWinBinCap) return false;   // uniform
    const uint32_t want = h[b];
    const uint32_t lo = wk + ((uint32_t)b << kWinShift);
    // the bin's keys (their low bits) into LDS: one wave-aggregated append per 64 keys;
    // kWinBatch 16-B loads per thread in flight before any is used (one at a time, the
    // walk over 36k keys was ~9 dependent round trips: K3 16 us at 1B)
    constexpr int kWinBatch = 8;
    const int64_t n4 = cnt / 4;
    const float4* x4 = reinterpret_cast<const float4*>(x);   // the window is 16-B aligned
    auto take = [&](float v) {
        const uint32_t d = __float_as_uint(v) - lo;   // v < 0 (padding): huge
        const bool in = v >= 0.f && d < (1u << kWinShift);
        const uint64_t m = __ballot(in);
        if (!m) return;
        const int leader = __ffsll((unsigned long long)m) - 1;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&nbuf, (uint32_t)__popcll(m));
        base = __shfl(base, leader);
        const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
        if (in && pos < (uint32_t)kWinBinCap) buf[pos] = d;
    };
    for (int64_t jb = 0; jb < n4; jb += kWinBatch * kScanThreads) {   // (the same trip count everywhere)
        float4 f[kWinBatch];
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            const int64_t j = jb + tid + (int64_t)u * kScanThreads;
            f[u] = j < n4 ? x4[j] : make_float4(-1.f, -1.f, -1.f, -1.f);
        }
#pragma unroll
        for (int u = 0; u < kWinBatch; ++u) {
            take(f[u].x);
            take(f[u].y);
            take(f[u].z);
            take(f[u].w);
        }
    }
    if (tid < (int)(cnt & 3u)) take(x[4 * n4 + tid]);   // (wave 0 only: its ballot is its own)
    __syncthreads();
    const uint32_t nb = nbuf;
    if (nb != want) return false;   // (cannot happen for a complete window) uniform
    for (int q = tid; q < (1 << kWinShift); q += kScanThreads) h[q] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < nb; i += kScanThreads) atomicAdd(&h[buf[i]], 1u);
    if (tid == 0) sel_bin = -1;
    __syncthreads();
    static_assert((1 << kWinShift) == kScanThreads, "one sub-bin per thread");
    if (pick_bin_small<1>(h, k - a, lds32, &bin, &above)) sel_bin = bin;
    __syncthreads();
    const int sb = sel_bin;
    if (tid == 0 && sb >= 0) *out = __uint_as_float(lo + (uint32_t)sb);
    __syncthreads();
    return sb >= 0;
}

__global__ void __launch_bounds__(kScanThreads)
k_rs_small(const float* __restrict__ x, int64_t n, uint64_t k, float* out) {
    rs_small_wg(x, n, k, out);
}

template <class Src>
__global__ void __launch_bounds__(kBlock) k_rs_hist(Src src, int pass) {
    rs_hist_body(src, pass, (int)blockIdx.x);
}

// The three passes in ONE launch (a source with chain words, src.chain(): 128 words,
// zero at rest): when no task is active — every window was selected in one workgroup, the
// steady state — every workgroup returns at once (three gated launches were ~15 us of a
// flat-1B step). Otherwise the passes run in order over virtual blocks claimed from an
// atomic counter, a workgroup waiting for a pass's completion count (chain_phase_end:
// one L2 write-back per XCD and pass, an acquire per workgroup); only running
// workgroups claim blocks, so nothing assumes the grid co-resident. The last workgroup
// out re-zeroes the words.
template <class Src>
__global__ void __launch_bounds__(kBlock) k_rs_passes(Src src, int grid, int ntasks) {
    __shared__ uint32_t s_u;
    bool mine_any = false;   // a task with blocks that the one-workgroup selections left to the passes
    for (int t = threadIdx.x; t < ntasks; t += blockDim.x) mine_any |= src.blocks(t) > 0 && src.active(t);
    if (!__syncthreads_or(mine_any)) return;   // uniform; no task turns active during the call
    uint32_t* cc = src.chain();   // [0..2] claims, [3] workgroups out; a ChainPhase per pass from word 32
#pragma unroll 1   // (unrolled, the three passes' bodies took 156 VGPRs: 3 waves per SIMD against 7)
    for (int pass = 0; pass < 3; ++pass) {
        uint32_t mine = 0;
        for (;;) {
            __syncthreads();
            if (threadIdx.x == 0) s_u = atomicAdd(&cc[pass], 1u);
            __syncthreads();
            const uint32_t vb = s_u;
            if (vb >= (uint32_t)grid) break;   // uniform
            rs_hist_body(src, pass, (int)vb);
            ++mine;
        }
        chain_phase_end(reinterpret_cast<ChainPhase*>(cc + 32) + pass, mine, (uint32_t)grid);
    }
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&cc[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1)
        for (int i = 0; i < 32 + 3 * 32; ++i) __hip_atomic_store(&cc[i], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The three histogram passes over any task source; every active task's state must
// have been reset with its k (rs_reset).
template <class Src>
inline int radix_select_passes(const Src& src, int grid, hipStream_t s) {
    if (grid <= 0) return DGC_OK;
    for (int pass = 0; pass < 3; ++pass) {
        hipLaunchKernelGGL((k_rs_hist<Src>), dim3(grid), dim3(kBlock), 0, s, src, pass);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

}  // namespace dgc
