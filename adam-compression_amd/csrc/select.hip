// K4: selection — the `importance >= threshold` mask, `nonzero()`, the adaptation
// loop, resample, truncation, value gather, momentum masking and wire packing —
// plus the listing K1 of the fused compress.
//
// Reference: DGCCompressor._sparsify (dgc/compression.py:109-153),
// DGCSGDMemory.update (dgc/memory.py:72-77), compress's casts (dgc/compression.py:168-171),
// compress's call order (dgc/compression.py:155-172).
//
// Layout. vec is cut into SEGMENTS of 1024 elements; 1024 segments form a GROUP
// (the scan granule and one emit workgroup). Every segment owns a candidate list of
// kCap = 64 slots (u16 offset + the fp32 value, ascending) and two exact counts:
// seg_lcnt at the LIST threshold t_list (a list is complete iff seg_lcnt <= kCap; a
// spilled segment is re-read from vec when needed) and seg_cnt at the current
// threshold t_cur >= t_list.
//
// Speculative listing. The fused compress lists candidates INSIDE K1, at
// t_list = margin x (the previous call's final threshold), kept on device. When the
// sampled threshold comes out >= t_list — the steady state — every count and every
// selection is served from the lists and the separate 4 B/elem re-read of vec
// disappears; otherwise a full select pass at t_cur re-lists (t_list := t_cur).
// Results are identical either way: a list at t_list holds EVERY element >= t_list.
//
//   count pass   t_cur >= t_list: one thread per segment counts its list entries
//                >= t_cur (spilled segments: one wave re-reads 1024 elements);
//                t_cur < t_list: full select pass (16 non-temporal float4 loads in
//                flight per lane, ballot compaction, re-lists at t_cur).
//   decide       (1 workgroup): total count -> the reference's loop step
//                (ok / trunc / resample / lower / raise / exhausted) + scan of the
//                group totals. resample=True: the first "lower" hands over to ONE
//                multi-threshold pass; resample=False: a recount per step.
//   resample     radix select of the k-th largest candidate, per-segment greater /
//                tied counts, scans. Ties go to the lowest indices (see oracle).
//   emit         (1 workgroup per group, 4 segments per thread): ascending positions,
//                fp32/fp16 values, int64/int32 indices, masking writes.
//
// Everything is stream-ordered; in DGC_SYNC_DEVICE mode kernels that turn out to
// be unneeded early-exit on a device flag, so no host synchronisation happens.
#include "radix_select.hpp"
#include "introselect.hpp"

namespace dgc {

constexpr int kSeg = 1024;                      // elements per segment
constexpr int kCap = 64;                        // list slots per segment (6.25 %)
constexpr int kSegTiles = kSeg / (kWave * 4);   // 4 float4 per lane per segment
constexpr int kSuper = 4;                       // segments per wave in the full select pass
constexpr int kGroupSegs = 1024;                // segments per group (1M elements)
constexpr int kSegPerBlock4 = kBlock / kWave;        // 4 waves per workgroup
constexpr int kMaxLower = 16;                   // thresholds per multi-threshold pass
constexpr int kSpillShards = 64;
constexpr int kSpillDiv = 32;                   // lists dropped when > nseg/32 segments spill

enum { MODE_FIRSTK = 0, MODE_RESAMPLE = 1 };

struct SelState {
    float t0, t_cur, tk, t_list;
    int32_t branch, iter, recounts, active;
    long long n_cur;       // count at t_cur
    long long limit;       // FIRSTK: emit the first `limit` candidates
    long long n_greater;   // RESAMPLE: candidates > tk
    long long tie_quota;   // RESAMPLE: k - n_greater ties, lowest index first
    int32_t resample_pending, overflow, done, lower_pending;
    int32_t full_passes, list_spills, epoch;
    int32_t rs_nth;        // RESAMPLE served by the exact nth_element replay (K5)
    int32_t tie_rule;      // DGC_TIES_*: how the resample chose among boundary ties
    uint32_t tickets[4];
    // Segments whose K1 list overflowed, counted by K1 into slot [epoch & 1] (64
    // shards against atomic contention); k_sel_init reads it and zeroes the other
    // slot for the next call, k_sel_finish advances the epoch.
    uint32_t spill[2][kSpillShards];
    unsigned long long lower_cnt[kMaxLower + 1];   // counts at t_1..t_m (multi-threshold pass)
};

struct SelWS {
    SelState* st;
    RSState* rs;
    uint32_t* seg_lcnt;
    uint32_t* seg_cnt;
    uint32_t* seg_gt;
    uint32_t* seg_eq;
    uint16_t* lst_off;
    float* lst_val;
    unsigned long long* grp_cnt;   // grp_cnt, grp_gt, grp_eq: contiguous, zeroed by k_sel_init
    unsigned long long* grp_gt;
    unsigned long long* grp_eq;
    long long* grp_off;
    long long* grp_gt_off;
    long long* grp_eq_off;
    uint64_t* queue;       // K5: (|x| key << 32 | j) for the candidates j, ascending index order
    int64_t* cand_idx;     // K5: the candidates' element indices
    uint32_t* gpos_l;      // K5: pair slots of the global-memory partition passes
    uint32_t* gpos_r;
    int64_t nseg, ngrp;
    int64_t cand_cap;      // K5 serves resamples of up to cand_cap candidates
};

// Candidates the exact resample replays: torch's CPU topk runs nth_element while
// k * 64 > n (else partial_sort, which is not replayed), so at most 64k - 1 of them.
__host__ __device__ inline int64_t nth_cand_cap(int64_t numel, int64_t k) {
    const int64_t c = 64 * k - 1;
    return c < numel ? c : numel;
}

static SelWS carve_select(void* base, int64_t numel, int64_t k, size_t* bytes = nullptr) {
    SelWS w{};
    w.nseg = ceil_div(numel, kSeg);
    w.ngrp = ceil_div(w.nseg, kGroupSegs);
    Carver c(base);
    w.st = c.take<SelState>(1);
    w.rs = c.take<RSState>(1);
    w.grp_cnt = c.take<unsigned long long>(3 * w.ngrp);
    w.grp_gt = w.grp_cnt ? w.grp_cnt + w.ngrp : nullptr;
    w.grp_eq = w.grp_gt ? w.grp_gt + w.ngrp : nullptr;
    w.grp_off = c.take<long long>(w.ngrp);
    w.grp_gt_off = c.take<long long>(w.ngrp);
    w.grp_eq_off = c.take<long long>(w.ngrp);
    w.seg_lcnt = c.take<uint32_t>(w.nseg);
    w.seg_cnt = c.take<uint32_t>(w.nseg);
    w.seg_gt = c.take<uint32_t>(w.nseg);
    w.seg_eq = c.take<uint32_t>(w.nseg);
    w.lst_off = c.take<uint16_t>(w.nseg * kCap);
    w.lst_val = c.take<float>(w.nseg * kCap);
    w.cand_cap = nth_cand_cap(numel, k);
    w.queue = c.take<uint64_t>(w.cand_cap);
    w.cand_idx = c.take<int64_t>(w.cand_cap);
    w.gpos_l = c.take<uint32_t>(w.cand_cap / 2 + 1);
    w.gpos_r = c.take<uint32_t>(w.cand_cap / 2 + 1);
    if (bytes) *bytes = c.bytes();
    return w;
}

static size_t select_ws_bytes(int64_t numel, int64_t k) {
    size_t b = 0;
    carve_select(nullptr, numel, k, &b);
    return b;
}

// ------------------------------------------------------------------ tile helpers
// Lane holds elements e0..e0+3 of a 256-element tile (e0 = tile base + 4*lane).
template <bool ALIGNED>
__device__ __forceinline__ void load_tile(const float* __restrict__ v, int64_t n, int64_t e0,
                                          float (&x)[4], uint32_t& valid) {
    if (ALIGNED && e0 + 3 < n) {
        const float4 q = ld_nt(reinterpret_cast<const float4*>(v + e0));
        x[0] = q.x;
        x[1] = q.y;
        x[2] = q.z;
        x[3] = q.w;
        valid = 0xFu;
    } else {
        valid = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool ok = e0 + j < n;
            x[j] = ok ? v[e0 + j] : 0.f;
            valid |= (uint32_t)ok << j;
        }
    }
}

__device__ __forceinline__ uint32_t ge_mask(const float (&x)[4], uint32_t valid, float t) {
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) p |= (uint32_t)(fabsf(x[j]) >= t) << j;
    return p & valid;
}

// Append the lanes' flagged elements (element order 4*lane + j) to a segment list.
__device__ __forceinline__ void list_append(uint32_t p, const float (&x)[4], int tile_off, uint32_t& c,
                                            uint16_t* lo, float* lv) {
    if (__ballot(p != 0)) {
        uint32_t lb, tot;
        wave_prefix4(p, lb, tot);
        uint32_t r = c + lb;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (p & (1u << j)) {
                if (r < (uint32_t)kCap) {
                    lo[r] = (uint16_t)(tile_off + 4 * lane + j);
                    lv[r] = x[j];
                }
                ++r;
            }
        }
        c += tot;
    }
}

// Count of |x| >= t over one segment, re-read from vec by the calling wave.
__device__ uint32_t wave_count_segment(const float* __restrict__ vec, int64_t n, int64_t seg, float t) {
    const int lane = threadIdx.x & 63;
    uint32_t c = 0;
    for (int tile = 0; tile < kSegTiles; ++tile) {
        float x[4];
        uint32_t valid;
        load_tile<false>(vec, n, seg * kSeg + tile * 256 + 4 * lane, x, valid);
        c += __popc(ge_mask(x, valid, t));
    }
    return wave_sum(c);
}

// ------------------------------------------------------------------ K1 with lists
// K1 (compensate + strided sample, see compensate.hip) that also lists every
// element with |vec_new| >= t_list into its segment's list. One wave per segment:
// float4 index = 256*seg + 64*u + lane (u = 0..3), each instruction 1 KB contiguous;
// non-temporal loads and stores. seg_lcnt = exact count at t_list; the segment that
// holds the < 4-element scalar tail is marked spilled (re-read when needed).
template <bool NEST, bool SAMPLE>
__global__ void __launch_bounds__(kBlock)
k_compensate_list(const float4* __restrict__ g, float4* __restrict__ mmt, float4* __restrict__ vec, int64_t n,
                  float mom, SampleSpec sp, const float* __restrict__ tspec, SelWS w) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t seg = (int64_t)blockIdx.x * kSegPerBlock4 + wave;
    const int64_t n4 = n / 4;
    const float tl = tspec ? *tspec : __builtin_huge_valf();
    if (blockIdx.x == 0 && threadIdx.x == 0) w.st->t_list = tl;
    // waves past the last segment load nothing and list nothing (v >= n4 below), but
    // stay for the block barrier of the spill count
    int64_t q0 = 0, r0 = 0;
    if (SAMPLE) floor_divmod_fast(seg * kSeg - sp.start, sp.stride, sp.inv_stride, q0, r0);
    float4 gv[kSegTiles], mv[kSegTiles], vv[kSegTiles];
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) {
        const int64_t v = seg * (kSeg / 4) + u * 64 + lane;
        if (v < n4) {
            gv[u] = ld_nt(g + v);
            mv[u] = ld_nt(mmt + v);
            vv[u] = ld_nt(vec + v);
        }
    }
    uint32_t c = 0;
    uint16_t* lo = w.lst_off + seg * kCap;
    float* lv = w.lst_val + seg * kCap;
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) {
        const int64_t v = seg * (kSeg / 4) + u * 64 + lane;
        const bool ok = v < n4;
        float x[4] = {0.f, 0.f, 0.f, 0.f};
        if (ok) {
            x[0] = comp1<NEST, true>(gv[u].x, mv[u].x, vv[u].x, mom);
            x[1] = comp1<NEST, true>(gv[u].y, mv[u].y, vv[u].y, mom);
            x[2] = comp1<NEST, true>(gv[u].z, mv[u].z, vv[u].z, mom);
            x[3] = comp1<NEST, true>(gv[u].w, mv[u].w, vv[u].w, mom);
            st_nt(mmt + v, mv[u]);
            st_nt(vec + v, vv[u]);
            if (SAMPLE) {
                const uint32_t t = (uint32_t)r0 + 4u * (uint32_t)(u * 64 + lane);
                const uint32_t s32 = (uint32_t)sp.stride;
                uint32_t q1, r;
                divmod_u32(t, s32, sp.inv_stride_f, q1, r);
                const uint32_t j = r == 0 ? 0u : s32 - r;
                if (j < 4) {
                    const int64_t qi = q0 + q1 + (r == 0 ? 0 : 1);
                    if (qi >= 0 && qi < sp.count) sp.out[qi] = fabsf(x[j]);
                }
            }
        }
        list_append(ge_mask(x, ok ? 0xFu : 0u, tl), x, u * 256, c, lo, lv);
    }
    const bool spilled = c > (uint32_t)kCap;
    if (lane == 0 && seg < w.nseg) {
        const bool tail = (n & 3) && seg == w.nseg - 1;
        w.seg_lcnt[seg] = tail ? (uint32_t)(kCap + 1) : c;
    }
    // one atomic per workgroup with a spilled segment (shard by block)
    const uint64_t any = __ballot(spilled);
    __shared__ uint32_t nsp;
    if (threadIdx.x == 0) nsp = 0;
    __syncthreads();
    if (lane == 0 && any) atomicAdd(&nsp, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && nsp)
        atomicAdd(&w.st->spill[w.st->epoch & 1][blockIdx.x % kSpillShards], nsp);
}

__global__ void k_no_lists(SelWS w) {
    if (threadIdx.x == 0) w.st->t_list = __builtin_huge_valf();
}

// ------------------------------------------------------------------ state
__global__ void __launch_bounds__(kScanThreads) k_sel_init(SelWS w, const float* thr0, int keep_lists) {
    SelState* st = w.st;
    for (int64_t i = threadIdx.x; i < 3 * w.ngrp; i += blockDim.x) w.grp_cnt[i] = 0;
    __shared__ uint32_t spills;
    if (threadIdx.x == 0) spills = 0;
    __syncthreads();
    const int e = st->epoch & 1;
    if (threadIdx.x < kSpillShards) {
        const uint32_t v = st->spill[e][threadIdx.x];
        if (v) atomicAdd(&spills, v);
        st->spill[e ^ 1][threadIdx.x] = 0;   // slot of the next call's K1
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const float t = *thr0;
        st->t0 = t;
        st->t_cur = t;
        st->list_spills = keep_lists ? (int32_t)spills : 0;
        // no K1 lists, or too many overflowed lists to be worth serving: one full pass
        if (!keep_lists || (int64_t)spills * kSpillDiv > w.nseg) st->t_list = __builtin_huge_valf();
        st->tk = 0.f;
        st->branch = -1;
        st->n_cur = st->limit = st->n_greater = st->tie_quota = 0;
        st->iter = st->recounts = 0;
        st->active = 1;
        st->resample_pending = 0;
        st->overflow = 0;
        st->done = 0;
        st->lower_pending = 0;
        st->full_passes = 0;
        st->rs_nth = 0;
        st->tie_rule = DGC_TIES_NONE;
        for (int i = 0; i < 4; ++i) st->tickets[i] = 0;
        for (int i = 0; i <= kMaxLower; ++i) st->lower_cnt[i] = 0;
    }
}

// ------------------------------------------------------------------ count passes
// t_cur >= t_list: counts from the lists, one thread per segment; spilled
// segments are re-read by the block's waves. One atomic per block into its group.
__global__ void __launch_bounds__(kBlock)
k_count_lists(const float* __restrict__ vec, int64_t n, SelWS w) {
    const SelState* st = w.st;
    if (!st->active || !(st->t_cur >= st->t_list)) return;
    const float t = st->t_cur;
    __shared__ int spill[kBlock];
    __shared__ int nspill;
    __shared__ uint32_t bsum;
    if (threadIdx.x == 0) {
        nspill = 0;
        bsum = 0;
    }
    __syncthreads();
    const int64_t seg = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t c = 0;
    if (seg < w.nseg) {
        const uint32_t lc = w.seg_lcnt[seg];
        if (lc <= (uint32_t)kCap) {
            const float4* l4 = reinterpret_cast<const float4*>(w.lst_val + seg * kCap);
            float4 v[kCap / 4];
#pragma unroll
            for (int q = 0; q < kCap / 4; ++q)   // all loads issued before any use
                if ((uint32_t)(4 * q) < lc) v[q] = l4[q];
#pragma unroll
            for (int q = 0; q < kCap / 4; ++q) {
                const uint32_t e = 4 * q;
                if (e < lc)
                    c += (fabsf(v[q].x) >= t) + (e + 1 < lc && fabsf(v[q].y) >= t) +
                         (e + 2 < lc && fabsf(v[q].z) >= t) + (e + 3 < lc && fabsf(v[q].w) >= t);
            }
            w.seg_cnt[seg] = c;
        } else {
            spill[atomicAdd(&nspill, 1)] = threadIdx.x;
        }
    }
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(&bsum, c);
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    for (int q = wave; q < nspill; q += kSegPerBlock4) {
        const int64_t s2 = (int64_t)blockIdx.x * kBlock + spill[q];
        const uint32_t cs = wave_count_segment(vec, n, s2, t);
        if ((threadIdx.x & 63) == 0) {
            w.seg_cnt[s2] = cs;
            if (cs) atomicAdd(&bsum, cs);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && bsum)
        atomicAdd(&w.grp_cnt[((int64_t)blockIdx.x * kBlock) / kGroupSegs], (unsigned long long)bsum);
}

// t_cur < t_list: full select pass at t_cur — one wave per kSuper segments (16
// float4 loads in flight per lane), re-lists every segment; seg_lcnt = seg_cnt.
template <bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
k_select_pass(const float* __restrict__ vec, int64_t n, SelWS w) {
    const SelState* st = w.st;
    if (!st->active || st->t_cur >= st->t_list) return;
    const float t = st->t_cur;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kTiles = kSuper * kSegTiles;   // 16
    __shared__ uint32_t wcnt[kSegPerBlock4];
    __shared__ uint32_t wovf[kSegPerBlock4];
    const int64_t nsuper = ceil_div(w.nseg, (int64_t)kSuper);
    // one-shot (grid = nsuper/4) or grid-stride with a capped grid (gated launches)
    for (int64_t bi = blockIdx.x; bi * kSegPerBlock4 < nsuper; bi += gridDim.x) {
        const int64_t sup = bi * kSegPerBlock4 + wave;
        uint32_t ctot = 0, novf = 0;
        if (sup < nsuper) {
            float x[kTiles][4];
            uint32_t valid[kTiles];
#pragma unroll
            for (int u = 0; u < kTiles; ++u)
                load_tile<ALIGNED>(vec, n, sup * (kSuper * kSeg) + u * 256 + 4 * lane, x[u], valid[u]);
#pragma unroll
            for (int sg = 0; sg < kSuper; ++sg) {
                const int64_t seg = sup * kSuper + sg;
                uint32_t c = 0;
                uint16_t* lo = w.lst_off + seg * kCap;
                float* lv = w.lst_val + seg * kCap;
#pragma unroll
                for (int u = 0; u < kSegTiles; ++u)
                    list_append(ge_mask(x[sg * kSegTiles + u], valid[sg * kSegTiles + u], t), x[sg * kSegTiles + u],
                                u * 256, c, lo, lv);
                if (lane == 0 && seg < w.nseg) {
                    w.seg_lcnt[seg] = c;
                    w.seg_cnt[seg] = c;
                }
                ctot += c;
                novf += c > (uint32_t)kCap;
            }
        }
        if (lane == 0) {
            wcnt[wave] = ctot;
            wovf[wave] = novf;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t s = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
            const uint32_t o = wovf[0] + wovf[1] + wovf[2] + wovf[3];
            if (s) atomicAdd(&w.grp_cnt[(bi * kSegPerBlock4 * kSuper) / kGroupSegs], (unsigned long long)s);
            if (o) atomicAdd(&w.st->overflow, (int)o);
        }
        __syncthreads();
    }
}

// Chunked exclusive scan of a[0..m) into out[] by one workgroup; returns the total.
// a[] holds totals accumulated by device atomics: read with agent-scope loads.
__device__ uint64_t block_scan_array(const unsigned long long* a, long long* out, int64_t m,
                                     uint64_t* lds16) {
    const int64_t per = ceil_div(m, (int64_t)blockDim.x);
    const int64_t b = threadIdx.x * per, e = b + per < m ? b + per : m;
    uint64_t local = 0;
    for (int64_t i = b; i < e; ++i) local += load_count(&a[i]);
    uint64_t total;
    uint64_t run = block_exclusive_scan(local, lds16, &total);
    for (int64_t i = b; i < e; ++i) {
        out[i] = (long long)run;
        run += load_count(&a[i]);
    }
    return total;
}

// One step of the reference's adaptation loop (dgc/compression.py:128-149) on the
// count of the pass that just ran. With resample (the default) the loop can only
// lower the threshold until the count reaches lower*k, so the first "lower" step
// hands over to ONE multi-threshold pass (k_lower_counts) instead of recounting
// one threshold per pass; without resample the threshold may also rise, and each
// step is a recount (count pass + decide), exactly like the reference.
__global__ void __launch_bounds__(kScanThreads)
k_decide(SelWS w, dgc_select_params p) {
    SelState* st = w.st;
    if (!st->active) return;
    __shared__ uint64_t lds16[16];
    __shared__ int finished, reset_rs;
    uint64_t local = 0;
    for (int64_t i = threadIdx.x; i < w.ngrp; i += kScanThreads) local += w.grp_cnt[i];
    uint64_t n;
    block_exclusive_scan(local, lds16, &n);
    if (threadIdx.x == 0) {
        if (st->t_cur < st->t_list) {   // a full select pass just re-listed at t_cur
            st->t_list = st->t_cur;
            st->full_passes += 1;
        }
        const long long cnt = (long long)n, k = p.num_selects;
        const bool adapt = p.numel > p.num_samples;
        st->n_cur = cnt;
        int done = 1;
        reset_rs = 0;
        if (!adapt) {
            st->branch = DGC_BRANCH_DIRECT;
            st->limit = cnt < k ? cnt : k;
        } else if (st->iter >= p.max_iters) {
            st->branch = DGC_BRANCH_EXHAUSTED;
            st->limit = cnt < k ? cnt : k;
        } else if (cnt > k) {
            if (cnt > p.upper_count) {
                if (p.resample) {
                    st->branch = DGC_BRANCH_RESAMPLE;
                    if (cnt < 64 * k && cnt <= w.cand_cap) {   // torch's nth_element path: replayed
                        st->rs_nth = 1;
                        st->tie_rule = DGC_TIES_EXACT;
                    } else {                                    // partial_sort path: lowest-index ties
                        st->resample_pending = 1;
                        st->tie_rule = DGC_TIES_LOWEST_INDEX;
                        reset_rs = 1;
                    }
                } else {
                    st->t_cur = __fmul_rn(st->t_cur, p.upper);
                    done = 0;
                }
            } else {
                st->branch = DGC_BRANCH_TRUNC;
                st->limit = k;
            }
        } else if (cnt < p.lower_count) {
            if (p.resample && st->iter == 0 && p.max_iters <= kMaxLower) {
                st->lower_pending = 1;   // k_lower_counts finds the final threshold in one pass
                done = 2;
            } else {
                st->t_cur = __fmul_rn(st->t_cur, p.lower);
                done = 0;
            }
        } else {
            st->branch = DGC_BRANCH_OK;
            st->limit = cnt;
        }
        if (done == 0) {
            st->iter += 1;
            st->recounts += 1;
            st->overflow = 0;
        } else if (done == 1) {
            st->active = 0;
            st->done = 1;
        } else {
            st->active = 0;
        }
        finished = done;
    }
    __syncthreads();
    if (finished == 1) block_scan_array(w.grp_cnt, w.grp_off, w.ngrp, lds16);
    if (reset_rs) rs_reset(w.rs, (uint64_t)p.num_selects);
    __syncthreads();
    if (finished != 1)
        for (int64_t i = threadIdx.x; i < w.ngrp; i += kScanThreads) w.grp_cnt[i] = 0;
}

// Counts at t_j = fl32(t_{j-1} * lower), j = 1..max_iters, in ONE pass over vec (the
// reference's "lower" recounts, dgc/compression.py:140-148, all at once). The last
// workgroup to arrive picks j* = the first j whose count reaches lower*k (else
// max_iters) and arms the count pass + decide at t_{j*}.
template <bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
k_lower_counts(const float* __restrict__ vec, int64_t n, SelWS w, dgc_select_params p) {
    SelState* st = w.st;
    if (!st->lower_pending) return;
    const int m = p.max_iters;
    float t[kMaxLower + 1];
    t[0] = st->t_cur;
#pragma unroll
    for (int j = 1; j <= kMaxLower; ++j) t[j] = __fmul_rn(t[j - 1], p.lower);
    const float tmin = t[m];
    uint32_t c[kMaxLower + 1];
#pragma unroll
    for (int j = 0; j <= kMaxLower; ++j) c[j] = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t seg = (int64_t)blockIdx.x * kSegPerBlock4 + wave; seg < w.nseg;
         seg += (int64_t)gridDim.x * kSegPerBlock4) {
        for (int tile = 0; tile < kSegTiles; ++tile) {
            float x[4];
            uint32_t valid;
            load_tile<ALIGNED>(vec, n, seg * kSeg + tile * 256 + 4 * lane, x, valid);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float a = fabsf(x[q]);
                if (((valid >> q) & 1u) && a >= tmin) {
#pragma unroll
                    for (int j = 1; j <= kMaxLower; ++j) c[j] += (j <= m) && a >= t[j];
                }
            }
        }
    }
    __shared__ uint32_t part[kSegPerBlock4][kMaxLower + 1];
#pragma unroll
    for (int j = 1; j <= kMaxLower; ++j) {
        const uint32_t v = wave_sum(c[j]);
        if (lane == 0) part[wave][j] = v;
    }
    __syncthreads();
    if (threadIdx.x >= 1 && threadIdx.x <= m) {
        const int j = threadIdx.x;
        const uint64_t v = (uint64_t)part[0][j] + part[1][j] + part[2][j] + part[3][j];
        if (v) atomicAdd(&st->lower_cnt[j], (unsigned long long)v);
    }
    if (!last_block_arrival(&st->tickets[0], gridDim.x)) return;
    if (threadIdx.x == 0) {
        int js = m;
        for (int j = 1; j <= m; ++j) {
            const long long nj = (long long)load_count(&st->lower_cnt[j]);
            if (nj >= p.lower_count) {
                js = j;
                break;
            }
        }
        st->t_cur = t[js];
        st->iter = js;
        st->recounts = js;
        st->overflow = 0;
        st->lower_pending = 0;
        st->active = 1;   // count pass + decide at t_{j*}
    }
}

// ------------------------------------------------------------------ resample
// Candidate keys (|x| >= t_cur) for the resample radix select: the segment list
// when complete, a re-read of vec when it spilled. One wave per segment.
struct CandKeys {
    const float* vec;
    int64_t n;
    SelWS w;
    template <class F>
    __device__ __forceinline__ void visit(F&& f) const {
        const int lane = threadIdx.x & 63;
        const int64_t gw = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
        const float t = w.st->t_cur;
        for (int64_t seg = gw; seg < w.nseg; seg += nw) {
            const uint32_t lc = w.seg_lcnt[seg];
            if (lc <= (uint32_t)kCap) {
                if (lane < lc) {
                    const float a = fabsf(w.lst_val[seg * kCap + lane]);
                    if (a >= t) f(abs_key(a));
                }
            } else {
                for (int tile = 0; tile < kSegTiles; ++tile) {
                    float x[4];
                    uint32_t valid;
                    load_tile<false>(vec, n, seg * kSeg + tile * 256 + 4 * lane, x, valid);
                    const uint32_t p = ge_mask(x, valid, t);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (p & (1u << j)) f(abs_key(x[j]));
                }
            }
        }
    }
};

// Per-segment counts of |x| > tk and |x| == tk (both imply |x| >= t_cur), one
// thread per segment, spilled segments re-read by waves; the last workgroup scans
// the group totals and sets the tie quota k - #greater.
__global__ void __launch_bounds__(kBlock)
k_count_gt_eq(const float* __restrict__ vec, int64_t n, SelWS w, int64_t k) {
    SelState* st = w.st;
    if (!st->resample_pending) return;
    const float tk = st->tk;
    __shared__ int spill[kBlock];
    __shared__ int nspill;
    __shared__ uint32_t bgt, beq;
    if (threadIdx.x == 0) {
        nspill = 0;
        bgt = beq = 0;
    }
    __syncthreads();
    const int64_t seg = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t gt = 0, eq = 0;
    if (seg < w.nseg) {
        const uint32_t lc = w.seg_lcnt[seg];
        if (lc <= (uint32_t)kCap) {
            for (uint32_t e = 0; e < lc; ++e) {
                const float a = fabsf(w.lst_val[seg * kCap + e]);
                gt += a > tk;
                eq += a == tk;
            }
            w.seg_gt[seg] = gt;
            w.seg_eq[seg] = eq;
        } else {
            spill[atomicAdd(&nspill, 1)] = threadIdx.x;
        }
    }
    gt = wave_sum(gt);
    eq = wave_sum(eq);
    if ((threadIdx.x & 63) == 0) {
        if (gt) atomicAdd(&bgt, gt);
        if (eq) atomicAdd(&beq, eq);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int q = wave; q < nspill; q += kSegPerBlock4) {
        const int64_t s2 = (int64_t)blockIdx.x * kBlock + spill[q];
        uint32_t g2 = 0, e2 = 0;
        for (int tile = 0; tile < kSegTiles; ++tile) {
            float x[4];
            uint32_t valid;
            load_tile<false>(vec, n, s2 * kSeg + tile * 256 + 4 * lane, x, valid);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a = fabsf(x[j]);
                const bool ok = (valid >> j) & 1u;
                g2 += ok && a > tk;
                e2 += ok && a == tk;
            }
        }
        g2 = wave_sum(g2);
        e2 = wave_sum(e2);
        if (lane == 0) {
            w.seg_gt[s2] = g2;
            w.seg_eq[s2] = e2;
            if (g2) atomicAdd(&bgt, g2);
            if (e2) atomicAdd(&beq, e2);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int64_t g = ((int64_t)blockIdx.x * kBlock) / kGroupSegs;
        if (bgt) atomicAdd(&w.grp_gt[g], (unsigned long long)bgt);
        if (beq) atomicAdd(&w.grp_eq[g], (unsigned long long)beq);
    }
    if (!last_block_arrival(&st->tickets[1], gridDim.x)) return;
    __shared__ uint64_t lds16[16];
    const uint64_t G = block_scan_array(w.grp_gt, w.grp_gt_off, w.ngrp, lds16);
    __syncthreads();
    block_scan_array(w.grp_eq, w.grp_eq_off, w.ngrp, lds16);
    if (threadIdx.x == 0) {
        st->n_greater = (long long)G;
        st->tie_quota = k - (long long)G;
        st->limit = k;
    }
}

// ------------------------------------------------------------------ emit
struct EmitOut {
    float* vec;          // null: leave vec untouched (pure selection)
    float* mmt;          // null: no momentum masking
    void* values;
    void* indices;
    int32_t vdtype, idtype;
    uint64_t* queue;     // non-null: K5 candidate gather (queue[pos] = key << 32 | pos, cand[pos] = index)
    int64_t* cand;
};

__device__ __forceinline__ void emit_one(const EmitOut& o, int64_t pos, int64_t gidx, float x) {
    if (o.queue) {
        o.queue[pos] = ((uint64_t)abs_key(x) << 32) | (uint64_t)(uint32_t)pos;
        o.cand[pos] = gidx;
        return;
    }
    store_value(o.values, pos, x, o.vdtype);
    store_index(o.indices, pos, gidx, o.idtype);
    // scattered 4-B writes, one per 128-B line: non-temporal (no L2 allocation)
    if (o.vec) __builtin_nontemporal_store(0.f, o.vec + gidx);
    if (o.mmt) __builtin_nontemporal_store(0.f, o.mmt + gidx);
}

// Wave-cooperative emit of one spilled segment by re-reading vec.
// FIRSTK: positions base + rank for |x| >= t, kept while < limit.
__device__ void emit_reread_firstk(const float* __restrict__ vec_in, int64_t n, int64_t seg, long long base,
                                   long long limit, float t, const EmitOut& o) {
    const int lane = threadIdx.x & 63;
    uint32_t run = 0;
    for (int tile = 0; tile < kSegTiles; ++tile) {
        float x[4];
        uint32_t valid;
        const int64_t e0 = seg * kSeg + tile * 256 + 4 * lane;
        load_tile<false>(vec_in, n, e0, x, valid);
        const uint32_t p = ge_mask(x, valid, t);
        if (__ballot(p != 0)) {
            uint32_t lb, tot;
            wave_prefix4(p, lb, tot);
            uint32_t r = run + lb;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (p & (1u << j)) {
                    const long long pos = base + r;
                    if (pos < limit) emit_one(o, pos, e0 + j, x[j]);
                    ++r;
                }
            run += tot;
        }
    }
}

// RESAMPLE: |x| > tk always, |x| == tk while the running tie rank is below T.
__device__ void emit_reread_resample(const float* __restrict__ vec_in, int64_t n, int64_t seg, long long bg,
                                     long long bt, float tk, long long T, const EmitOut& o) {
    const int lane = threadIdx.x & 63;
    uint32_t run_g = 0, run_t = 0;
    for (int tile = 0; tile < kSegTiles; ++tile) {
        float x[4];
        uint32_t valid;
        const int64_t e0 = seg * kSeg + tile * 256 + 4 * lane;
        load_tile<false>(vec_in, n, e0, x, valid);
        uint32_t pg = 0, pe = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a = fabsf(x[j]);
            pg |= (uint32_t)(a > tk) << j;
            pe |= (uint32_t)(a == tk) << j;
        }
        pg &= valid;
        pe &= valid;
        if (__ballot((pg | pe) != 0)) {
            uint32_t lg, tg, lt, tt;
            wave_prefix4(pg, lg, tg);
            wave_prefix4(pe, lt, tt);
            uint32_t rg = run_g + lg, rt = run_t + lt;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool gt = (pg >> j) & 1u, eq = (pe >> j) & 1u;
                const long long tb = bt + rt;
                if (gt || (eq && tb < T)) emit_one(o, bg + rg + (tb < T ? tb : T), e0 + j, x[j]);
                rg += gt;
                rt += eq;
            }
            run_g += tg;
            run_t += tt;
        }
    }
}

// One workgroup per group of kGroupSegs segments, one thread per segment for the
// in-group offset scan; then wave-per-segment emission: kCap == 64 list slots, so
// lane l takes list entry l (one coalesced load per list) and ballot ranks give the
// output positions. Each wave emits 64 consecutive segments, kEmitBatch lists in
// flight; a spilled segment is re-read from vec by the same wave.
constexpr int kEmitThreads = kGroupSegs;
constexpr int kEmitBatch = 8;
constexpr uint32_t kEmitSkip = 0xFFFFFFFFu;
static_assert(kCap == kWave, "wave-per-list emission needs kCap == wavefront width");

// o.queue == null: the payload (every branch but a K5 resample, which k_emit_queue
// writes). o.queue != null: K5's candidate gather — every element >= t_cur, ascending
// (the reference's `indices` before its resample topk), only when K5 serves the step.
__global__ void __launch_bounds__(kEmitThreads)
k_emit(const float* __restrict__ vec_in, int64_t n, SelWS w, EmitOut o) {
    const SelState* st = w.st;
    const bool k5 = st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth;
    if (k5 != (o.queue != nullptr)) return;
    const bool rs = st->branch == DGC_BRANCH_RESAMPLE && !k5;
    const int64_t g = blockIdx.x;
    const int64_t seg0 = g * kGroupSegs;
    __shared__ uint32_t off_a[kGroupSegs], off_b[kGroupSegs], lcn[kGroupSegs];
    __shared__ uint64_t lds16[16];
    const long long limit = k5 ? st->n_cur : st->limit;
    const long long T = st->tie_quota;
    const long long ga = rs ? w.grp_gt_off[g] : w.grp_off[g];
    const long long gb = rs ? w.grp_eq_off[g] : 0;
    {
        const int64_t seg = seg0 + threadIdx.x;
        uint32_t ca = 0, cb = 0, lc = 0;
        if (seg < w.nseg) {
            ca = rs ? w.seg_gt[seg] : w.seg_cnt[seg];
            cb = rs ? w.seg_eq[seg] : 0;
            lc = w.seg_lcnt[seg];
        }
        uint64_t tot;
        const uint32_t oa = (uint32_t)block_exclusive_scan((uint64_t)ca, lds16, &tot);
        __syncthreads();
        const uint32_t ob = rs ? (uint32_t)block_exclusive_scan((uint64_t)cb, lds16, &tot) : 0u;
        const bool work = rs ? (ca > 0 || (cb > 0 && gb + ob < T)) : (ca > 0 && ga + oa < limit);
        off_a[threadIdx.x] = oa;
        off_b[threadIdx.x] = ob;
        lcn[threadIdx.x] = work ? lc : kEmitSkip;
    }
    __syncthreads();
    const float t = st->t_cur, tk = st->tk;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    for (int j0 = wv * 64; j0 < wv * 64 + 64; j0 += kEmitBatch) {
        float x[kEmitBatch];
        uint32_t e[kEmitBatch];
#pragma unroll
        for (int q = 0; q < kEmitBatch; ++q) {   // all list loads issued first
            const uint32_t L = lcn[j0 + q];
            x[q] = 0.f;
            e[q] = 0;
            if (L <= (uint32_t)kCap && (uint32_t)lane < L) {
                const int64_t slot = (seg0 + j0 + q) * kCap + lane;
                x[q] = w.lst_val[slot];
                e[q] = w.lst_off[slot];
            }
        }
#pragma unroll
        for (int q = 0; q < kEmitBatch; ++q) {
            const uint32_t L = lcn[j0 + q];
            if (L == kEmitSkip) continue;
            const int64_t seg = seg0 + j0 + q;
            const long long ba = ga + off_a[j0 + q], bb = gb + off_b[j0 + q];
            if (L > (uint32_t)kCap) {
                if (rs)
                    emit_reread_resample(vec_in, n, seg, ba, bb, tk, T, o);
                else
                    emit_reread_firstk(vec_in, n, seg, ba, limit, t, o);
                continue;
            }
            const bool in = (uint32_t)lane < L;
            const float a = fabsf(x[q]);
            const int64_t gidx = seg * kSeg + e[q];
            if (!rs) {
                const bool sel = in && a >= t;
                const uint64_t m = __ballot(sel);
                const long long pos = ba + __popcll(m & lt);
                if (sel && pos < limit) emit_one(o, pos, gidx, x[q]);
            } else {
                const bool gt = in && a > tk, eq = in && a == tk;
                const uint64_t mg = __ballot(gt), me = __ballot(eq);
                const long long tb = bb + __popcll(me & lt);
                if (gt || (eq && tb < T)) emit_one(o, ba + __popcll(mg & lt) + (tb < T ? tb : T), gidx, x[q]);
            }
        }
    }
}

// K5: the reference's resample topk replayed on the gathered candidates (introselect.hpp).
__global__ void __launch_bounds__(kNthThreads) k_nth_select(SelWS w, int64_t k) {
    const SelState* st = w.st;
    if (!(st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth)) return;
    nth_element_wg(w.queue, st->n_cur, k - 1, w.gpos_l, w.gpos_r);
}

// K5 emit: output slot q <- candidate queue[q] (the topk's order), with values,
// wire casts and the masking of DGCSGDMemory.update.
__global__ void __launch_bounds__(kBlock) k_emit_queue(const float* __restrict__ vec_in, SelWS w, EmitOut o,
                                                      int64_t k) {
    const SelState* st = w.st;
    if (!(st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth)) return;
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < k; q += (int64_t)gridDim.x * kBlock) {
        const uint32_t j = (uint32_t)w.queue[q];
        const int64_t gidx = w.cand_idx[j];
        emit_one(o, q, gidx, vec_in[gidx]);
    }
}

// Result record; and the next call's speculative list threshold, margin x t_cur.
__global__ void k_sel_finish(SelState* st, int64_t k, int64_t* count_out, dgc_select_info* info,
                             float* spec, float margin) {
    if (threadIdx.x != 0) return;
    st->epoch += 1;
    const long long cnt = st->branch == DGC_BRANCH_RESAMPLE ? k : st->limit;
    if (count_out) *count_out = cnt;
    if (info) {
        info->count = cnt;
        info->candidates = st->n_cur;
        info->threshold0 = st->t0;
        info->threshold = st->t_cur;
        info->branch = st->branch;
        info->recounts = st->recounts;
        info->overflow_segments = st->full_passes ? st->overflow : st->list_spills;
        info->full_passes = st->full_passes;
        info->tie_rule = st->tie_rule;
        info->pad = 0;
    }
    if (spec) {
        // spec[0]: next call's list threshold = margin * t * growth, growth = t / spec[1]
        // (the previous final threshold) clamped to [1, 1.5]; spec[1] := t.
        const float t = st->t_cur;
        const float g = fminf(fmaxf(t / spec[1], 1.f), 1.5f);   // NaN (first call: inf/inf) -> 1
        spec[0] = (t == t && t > 0.f && t < __builtin_huge_valf()) ? t * margin * g : __builtin_huge_valf();
        spec[1] = t;
    }
}

// ------------------------------------------------------------------ host driver
static int validate_select(const dgc_select_params* p, void* values, void* indices) {
    if (!p) DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null params");
    if (p->numel < 1 || p->num_selects < 1 || p->num_selects > p->numel)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: need 1 <= num_selects <= numel (got %lld, %lld)",
                 (long long)p->num_selects, (long long)p->numel);
    if (p->num_samples < 1 || p->num_samples > p->numel)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: bad num_samples");
    if (p->max_iters < 0) DGC_FAIL(DGC_ERR_INVALID, "dgc_select: max_iters < 0");
    if (p->vdtype != DGC_F32 && p->vdtype != DGC_F16) DGC_FAIL(DGC_ERR_DTYPE, "dgc_select: value dtype");
    if (p->idtype != DGC_I64 && p->idtype != DGC_I32) DGC_FAIL(DGC_ERR_DTYPE, "dgc_select: index dtype");
    if (p->idtype == DGC_I32 && p->numel > 2147483647LL)
        DGC_FAIL(DGC_ERR_OVERFLOW, "dgc_select: int32 indices cannot address %lld elements",
                 (long long)p->numel);
    if (!values || !indices) DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null outputs");
    return DGC_OK;
}

// Selection on an already-carved workspace. keep_lists: the lists / seg_lcnt /
// t_list in the workspace are valid (written by the listing K1).
static int select_core(float* vec, float* mmt, const float* thr0, const dgc_select_params* p, void* values,
                       void* indices, int64_t* count_out, dgc_select_info* info, const SelWS& w, int keep_lists,
                       int sync_mode, float* spec, float margin, hipStream_t s) {
    const int64_t n = p->numel;
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(kScanThreads), 0, s, w, thr0, keep_lists);
    DGC_LAUNCHED();
    const int64_t nsuper = ceil_div(w.nseg, (int64_t)kSuper);
    const int grid_full = (int)ceil_div(nsuper, kSegPerBlock4);   // one-shot full pass
    const int grid_gs = grid_for(nsuper, kSegPerBlock4);          // grid-stride (gated) kernels
    const int grid_cl = (int)ceil_div(w.nseg, kBlock);           // list count: a thread per segment
    const bool al = aligned16(vec);
    const bool adapt = p->numel > p->num_samples;
    const bool lower_fast = p->resample && p->max_iters <= kMaxLower;
    // One count pass at t_cur: k_count_lists serves t_cur >= t_list from the lists,
    // k_select_pass re-reads vec (and re-lists) below it. Both are gated on the device;
    // `need` says which may run: 1 = lists only, 2 = full pass only, 3 = either.
    // The first pass of dgc_select (no K1 lists, t_list = inf) is always a full pass.
    auto pass = [&](int need, bool likely_lists) -> int {
        if (need & 1) {
            hipLaunchKernelGGL(k_count_lists, dim3(grid_cl), dim3(kBlock), 0, s, vec, n, w);
            DGC_LAUNCHED();
        }
        if (need & 2) {
            const int gf = likely_lists ? grid_gs : grid_full;
            if (al)
                hipLaunchKernelGGL(k_select_pass<true>, dim3(gf), dim3(kBlock), 0, s, vec, n, w);
            else
                hipLaunchKernelGGL(k_select_pass<false>, dim3(gf), dim3(kBlock), 0, s, vec, n, w);
            DGC_LAUNCHED();
        }
        hipLaunchKernelGGL(k_decide, dim3(1), dim3(kScanThreads), 0, s, w, *p);
        DGC_LAUNCHED();
        return DGC_OK;
    };
    auto lower = [&]() -> int {
        if (al)
            hipLaunchKernelGGL(k_lower_counts<true>, dim3(grid_gs), dim3(kBlock), 0, s, vec, n, w, *p);
        else
            hipLaunchKernelGGL(k_lower_counts<false>, dim3(grid_gs), dim3(kBlock), 0, s, vec, n, w, *p);
        DGC_LAUNCHED();
        return DGC_OK;
    };
    EmitOut o{p->update_memory ? vec : nullptr, (p->update_memory && p->masking) ? mmt : nullptr, values,
              indices, p->vdtype, p->idtype, nullptr, nullptr};
    auto resample_lowest = [&]() -> int {
        // partial_sort path (>= 64k candidates): radix k-th value, ties lowest index first.
        // rs state reset by k_decide when it chose this path
        CandKeys src{vec, n, w};
        DGC_TRY(radix_select_passes(src, grid_for(w.nseg, kSegPerBlock4), &w.st->tk, w.rs,
                                    &w.st->resample_pending, s));
        hipLaunchKernelGGL(k_count_gt_eq, dim3(grid_cl), dim3(kBlock), 0, s, vec, n, w, (int64_t)p->num_selects);
        DGC_LAUNCHED();
        return DGC_OK;
    };
    auto resample_exact = [&]() -> int {
        // nth_element path: gather candidates, replay the introselect, emit in its order
        EmitOut g = o;
        g.queue = w.queue;
        g.cand = w.cand_idx;
        hipLaunchKernelGGL(k_emit, dim3((unsigned)w.ngrp), dim3(kEmitThreads), 0, s, vec, n, w, g);
        DGC_LAUNCHED();
        hipLaunchKernelGGL(k_nth_select, dim3(1), dim3(kNthThreads), 0, s, w, (int64_t)p->num_selects);
        DGC_LAUNCHED();
        hipLaunchKernelGGL(k_emit_queue, dim3(grid_for(p->num_selects)), dim3(kBlock), 0, s, vec, w, o,
                           (int64_t)p->num_selects);
        DGC_LAUNCHED();
        return DGC_OK;
    };
    DGC_TRY(keep_lists ? pass(3, true) : pass(2, false));
    if (sync_mode == DGC_SYNC_HOST) {
        // read each decision back and launch only what it needs
        SelState hs{};
        for (;;) {
            DGC_HIP(hipMemcpyAsync(&hs, w.st, sizeof(hs), hipMemcpyDeviceToHost, s));
            DGC_HIP(hipStreamSynchronize(s));
            if (hs.done) break;
            if (hs.lower_pending) {
                DGC_TRY(lower());   // picks t_cur on the device: either pass may follow
                DGC_TRY(pass(3, false));
            } else {
                DGC_TRY(pass(hs.t_cur >= hs.t_list ? 1 : 2, false));
            }
        }
        if (hs.branch == DGC_BRANCH_RESAMPLE) DGC_TRY(hs.rs_nth ? resample_exact() : resample_lowest());
    } else if (adapt) {
        // every kernel below early-exits on a device flag when it is not needed
        if (lower_fast) {
            DGC_TRY(lower());
            DGC_TRY(pass(3, true));
        } else {
            for (int i = 0; i < p->max_iters; ++i) DGC_TRY(pass(3, true));
        }
        if (p->resample) {
            DGC_TRY(resample_lowest());
            DGC_TRY(resample_exact());
        }
    }
    hipLaunchKernelGGL(k_emit, dim3((unsigned)w.ngrp), dim3(kEmitThreads), 0, s, vec, n, w, o);
    DGC_LAUNCHED();
    hipLaunchKernelGGL(k_sel_finish, dim3(1), dim3(64), 0, s, w.st, (int64_t)p->num_selects, count_out, info,
                       spec, margin);
    DGC_LAUNCHED();
    return DGC_OK;
}

int select(float* vec, float* mmt, const float* thr0, const dgc_select_params* p, void* values,
           void* indices, int64_t* count_out, dgc_select_info* info, void* ws, size_t ws_bytes,
           int sync_mode, hipStream_t s) {
    DGC_TRY(validate_select(p, values, indices));
    if (!vec || !thr0 || (p->update_memory && p->masking && !mmt))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null vec/thr0/mmt");
    const int64_t n = p->numel;
    if (!ws || ws_bytes < select_ws_bytes(n, p->num_selects) || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_select: workspace needs %zu bytes, 256-B aligned",
                 select_ws_bytes(n, p->num_selects));
    SelWS w = carve_select(ws, n, p->num_selects);
    return select_core(vec, mmt, thr0, p, values, indices, count_out, info, w, 0, sync_mode, nullptr, 1.f, s);
}

// ------------------------------------------------------------------ threshold
static size_t kth_ws_bytes(int64_t n) { return n <= kSmallN ? 256 : align_up(sizeof(RSState), 256); }

int kth_largest(const float* x, int64_t n, int64_t k, float* out, void* ws, size_t ws_bytes, hipStream_t s) {
    if (!x || !out || n < 1 || k < 1 || k > n)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_kth_largest: need 1 <= k <= n (k=%lld n=%lld)", (long long)k,
                 (long long)n);
    if (n <= kSmallN) {
        hipLaunchKernelGGL(k_rs_small, dim3(1), dim3(kScanThreads), 0, s, x, n, (uint64_t)k, out);
        DGC_LAUNCHED();
        return DGC_OK;
    }
    if (!ws || ws_bytes < sizeof(RSState) || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_kth_largest: workspace needs %zu bytes", sizeof(RSState));
    return radix_select_launch(DenseKeys{x, n}, n, (uint64_t)k, out, reinterpret_cast<RSState*>(ws), s);
}

// ------------------------------------------------------------------ fused compress
int compensate(const float* grad, float* mmt, float* vec, float* out, int64_t n, float momentum,
               bool nesterov, bool accumulate, float* samples, int64_t s_start, int64_t s_stride,
               int64_t s_count, hipStream_t st);
int sample_strided_launch(const float* vec, int64_t start, int64_t stride, int64_t count, float* out,
                          hipStream_t s);

struct CompressWS {
    float* thr;
    float* samples;
    RSState* rs;
    void* sel;
    size_t sel_bytes;
};

// sample_buf: floats reserved for the strided samples (0 when numel == num_samples)
static CompressWS carve_compress(void* base, int64_t numel, int64_t k, int64_t sample_buf, size_t* bytes = nullptr) {
    Carver c(base);
    CompressWS w{};
    w.thr = c.take<float>(64);
    w.rs = c.take<RSState>(1);
    w.samples = c.take<float>(sample_buf);
    w.sel_bytes = select_ws_bytes(numel, k);
    w.sel = c.take<char>(w.sel_bytes);
    if (bytes) *bytes = c.bytes();
    return w;
}

static size_t compress_ws_bytes(int64_t numel, int64_t k, int64_t sample_buf) {
    size_t b = 0;
    carve_compress(nullptr, numel, k, sample_buf, &b);
    return b;
}

struct CompressArgs {
    int64_t n, L, sbuf;
    bool sampled;
};

static int compress_check(const dgc_select_params* p, void* values, void* indices, int64_t s_start,
                          int64_t s_stride, int64_t top_k_samples, void* ws, size_t ws_bytes, CompressArgs* a,
                          bool need_outputs) {
    if (need_outputs) DGC_TRY(validate_select(p, values, indices));
    else if (!p) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: null params");
    a->n = p->numel;
    a->sampled = p->numel != p->num_samples;
    if (a->sampled && (s_stride < 2 || s_start < 0 || s_start >= s_stride))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: sample_start must be in [0, stride)");
    a->L = a->sampled ? ceil_div(a->n - s_start, s_stride) : a->n;
    if (need_outputs && (top_k_samples < 1 || top_k_samples > a->L))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: top_k_samples %lld outside [1, %lld]",
                 (long long)top_k_samples, (long long)a->L);
    a->sbuf = a->sampled ? a->L : 0;
    if (!ws || ws_bytes < compress_ws_bytes(a->n, p->num_selects, a->sbuf) || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_compress: workspace needs %zu bytes, 256-B aligned",
                 compress_ws_bytes(a->n, p->num_selects, a->sbuf));
    return DGC_OK;
}

// K1 (+ fused strided sample + speculative candidate lists at *spec).
int compress_begin(const float* grad, float* mmt, float* vec, float momentum, bool nesterov, int64_t s_start,
                   int64_t s_stride, const dgc_select_params* p, const float* spec, void* ws, size_t ws_bytes,
                   hipStream_t s) {
    CompressArgs a{};
    DGC_TRY(compress_check(p, nullptr, nullptr, s_start, s_stride, 1, ws, ws_bytes, &a, false));
    if (!grad || !mmt || !vec) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: null grad/mmt/vec");
    CompressWS cw = carve_compress(ws, a.n, p->num_selects, a.sbuf);
    SelWS w = carve_select(cw.sel, a.n, p->num_selects);
    const bool list_path = aligned16(grad) && aligned16(mmt) && aligned16(vec) &&
                           (!a.sampled || (s_stride >= 4 && s_stride < (1LL << 30)));
    if (!list_path) {
        DGC_TRY(compensate(grad, mmt, vec, nullptr, a.n, momentum, nesterov, true, a.sampled ? cw.samples : nullptr,
                           s_start, s_stride, a.sampled ? a.L : 0, s));
        hipLaunchKernelGGL(k_no_lists, dim3(1), dim3(64), 0, s, w);
        DGC_LAUNCHED();
        return DGC_OK;
    }
    SampleSpec sp{a.sampled ? cw.samples : nullptr, s_start, s_stride, a.sampled ? a.L : 0,
                  1.0 / (double)s_stride, 1.0f / (float)s_stride};
    const int64_t grid = ceil_div(w.nseg, kSegPerBlock4);
    if (grid > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: n too large");
    auto g4 = reinterpret_cast<const float4*>(grad);
    auto m4 = reinterpret_cast<float4*>(mmt);
    auto v4 = reinterpret_cast<float4*>(vec);
    if (nesterov) {
        if (a.sampled)
            hipLaunchKernelGGL((k_compensate_list<true, true>), dim3((unsigned)grid), dim3(kBlock), 0, s, g4, m4, v4,
                               a.n, momentum, sp, spec, w);
        else
            hipLaunchKernelGGL((k_compensate_list<true, false>), dim3((unsigned)grid), dim3(kBlock), 0, s, g4, m4,
                               v4, a.n, momentum, sp, spec, w);
    } else {
        if (a.sampled)
            hipLaunchKernelGGL((k_compensate_list<false, true>), dim3((unsigned)grid), dim3(kBlock), 0, s, g4, m4,
                               v4, a.n, momentum, sp, spec, w);
        else
            hipLaunchKernelGGL((k_compensate_list<false, false>), dim3((unsigned)grid), dim3(kBlock), 0, s, g4, m4,
                               v4, a.n, momentum, sp, spec, w);
    }
    DGC_LAUNCHED();
    if (a.n & 3) {   // scalar tail (< 4 elements) incl. its samples; its segment is marked spilled
        const int64_t done = (a.n / 4) * 4;
        DGC_TRY(compensate(grad + done, mmt + done, vec + done, nullptr, a.n - done, momentum, nesterov, true,
                           nullptr, 0, 1, 0, s));
        if (a.sampled) {
            // samples in the tail: start + q*stride >= done
            const int64_t q_first = done >= s_start ? ceil_div(done - s_start, s_stride) : 0;
            const int64_t cnt = a.L - q_first;
            if (cnt > 0) {
                const int64_t st0 = s_start + q_first * s_stride;
                DGC_TRY(sample_strided_launch(vec, st0, s_stride, cnt, cw.samples + q_first, s));
            }
        }
    }
    return DGC_OK;
}

// K3 threshold over the samples, then the selection (lists kept from begin).
int compress_finish(float* vec, float* mmt, int64_t s_start, int64_t s_stride, int64_t top_k_samples,
                    const dgc_select_params* p, float* spec, float margin, void* values, void* indices,
                    int64_t* count_out, dgc_select_info* info, void* ws, size_t ws_bytes, int sync_mode,
                    hipStream_t s) {
    CompressArgs a{};
    DGC_TRY(compress_check(p, values, indices, s_start, s_stride, top_k_samples, ws, ws_bytes, &a, true));
    if (!vec || (p->masking && !mmt)) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: null vec/mmt");
    CompressWS cw = carve_compress(ws, a.n, p->num_selects, a.sbuf);
    const float* src = a.sampled ? cw.samples : vec;
    DGC_TRY(kth_largest(src, a.L, top_k_samples, cw.thr, cw.rs, sizeof(RSState), s));
    SelWS w = carve_select(cw.sel, a.n, p->num_selects);
    dgc_select_params q = *p;
    q.update_memory = 1;   // DGCSGDMemory.update fused into the emit
    return select_core(vec, mmt, cw.thr, &q, values, indices, count_out, info, w, 1, sync_mode, spec, margin, s);
}

}  // namespace dgc

// ------------------------------------------------------------------ C ABI
extern "C" size_t dgc_kth_largest_workspace(int64_t n) { return dgc::kth_ws_bytes(n); }

extern "C" int dgc_kth_largest(const float* x, int64_t n, int64_t k, float* thr_out, void* ws,
                               size_t ws_bytes, void* stream) {
    return dgc::kth_largest(x, n, k, thr_out, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" size_t dgc_select_workspace(int64_t numel, int64_t num_selects) {
    return dgc::select_ws_bytes(numel, num_selects);
}

extern "C" int dgc_select(float* vec, float* mmt, const float* thr0, const dgc_select_params* params,
                          void* values_out, void* indices_out, int64_t* count_out,
                          dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                          void* stream) {
    return dgc::select(vec, mmt, thr0, params, values_out, indices_out, count_out, info_out, ws, ws_bytes,
                       sync_mode, static_cast<hipStream_t>(stream));
}

extern "C" size_t dgc_compress_workspace(int64_t numel, int64_t num_selects, int64_t num_samples) {
    // the strided slice holds ceil((numel - start) / stride) <= num_samples + 1 samples
    return dgc::compress_ws_bytes(numel, num_selects, numel == num_samples ? 0 : num_samples + 1);
}

extern "C" int dgc_compress_begin(const float* grad, float* mmt, float* vec, float momentum, int32_t nesterov,
                                  int64_t sample_start, int64_t sample_stride, const dgc_select_params* params,
                                  const float* spec_threshold, void* ws, size_t ws_bytes, void* stream) {
    return dgc::compress_begin(grad, mmt, vec, momentum, nesterov != 0, sample_start, sample_stride, params,
                               spec_threshold, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_compress_finish(float* vec, float* mmt, int64_t sample_start, int64_t sample_stride,
                                   int64_t top_k_samples, const dgc_select_params* params, float* spec_threshold,
                                   float spec_margin, void* values_out, void* indices_out, int64_t* count_out,
                                   dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                                   void* stream) {
    return dgc::compress_finish(vec, mmt, sample_start, sample_stride, top_k_samples, params, spec_threshold,
                                spec_margin, values_out, indices_out, count_out, info_out, ws, ws_bytes,
                                sync_mode, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_compress(const float* grad, float* mmt, float* vec, float momentum, int32_t nesterov,
                            int64_t sample_start, int64_t sample_stride, int64_t top_k_samples,
                            const dgc_select_params* params, float* spec_threshold, float spec_margin,
                            void* values_out, void* indices_out, int64_t* count_out, dgc_select_info* info_out,
                            void* ws, size_t ws_bytes, int32_t sync_mode, void* stream) {
    int rc = dgc::compress_begin(grad, mmt, vec, momentum, nesterov != 0, sample_start, sample_stride, params,
                                 spec_threshold, ws, ws_bytes, static_cast<hipStream_t>(stream));
    if (rc != DGC_OK) return rc;
    return dgc::compress_finish(vec, mmt, sample_start, sample_stride, top_k_samples, params, spec_threshold,
                                spec_margin, values_out, indices_out, count_out, info_out, ws, ws_bytes,
                                sync_mode, static_cast<hipStream_t>(stream));
}
