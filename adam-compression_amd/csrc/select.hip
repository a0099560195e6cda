// K4: selection — the `importance >= threshold` mask, `nonzero()`, the adaptation
// loop, resample, truncation, value gather, momentum masking and wire packing.
//
// Reference: DGCCompressor._sparsify (dgc/compression.py:109-153),
// DGCSGDMemory.update (dgc/memory.py:72-77), compress's casts (dgc/compression.py:168-171).
//
// Layout. vec is cut into SEGMENTS of 4096 elements, one wavefront each; 256
// segments form a GROUP (the scan granule and one emit workgroup).
//
//   select pass  (1 read of vec, 4 B/elem): each wave streams its segment with
//                16-B loads, |x| >= t by 64-lane ballots, and appends candidates
//                (u16 offset + fp32 value) to the segment's list in ascending
//                order (capacity kCap); exact per-segment counts; one 64-bit atomic
//                per block into the group total.
//   decide       (1 workgroup): total count -> the reference's loop step
//                (ok / trunc / resample / lower / raise / exhausted), exclusive scan
//                of group totals. A recount re-runs the select pass at the new
//                threshold (the reference re-scans too); all decisions stay on device.
//   resample     radix select of the k-th largest candidate (candidate lists; a
//                spilled segment is re-read from vec), per-segment counts of
//                greater / tied, scan. Ties go to the lowest indices (see oracle).
//   emit         (1 workgroup per group): ascending output positions from the
//                scans, fp32/fp16 values, int64/int32 indices, and the masking
//                writes vec[i] = 0 (mmt[i] = 0 when momentum_masking).
//
// Everything is stream-ordered; in DGC_SYNC_DEVICE mode kernels that turn out to
// be unneeded early-exit on a device flag, so no host synchronisation happens.
#include "radix_select.hpp"

namespace dgc {

constexpr int kSeg = 4096;
constexpr int kSegPerBlock = kBlock / kWave;   // 4
constexpr int kCap = 256;
constexpr int kGroupSegs = 256;
constexpr int kTiles = kSeg / (kWave * 4);    // 16 float4 tiles per lane
#ifndef DGC_SEL_BATCH
#define DGC_SEL_BATCH 16
#endif
constexpr int kSelBatch = DGC_SEL_BATCH;       // tile loads in flight per lane

constexpr int kMaxLower = 16;                  // thresholds per multi-threshold pass

enum { MODE_FIRSTK = 0, MODE_RESAMPLE = 1 };

struct SelState {
    float t0, t_cur, tk;
    int32_t branch;
    long long n_cur;       // count at t_cur
    long long limit;       // FIRSTK: emit the first `limit` candidates
    long long n_greater;   // RESAMPLE: candidates > tk
    long long tie_quota;   // RESAMPLE: k - n_greater ties, lowest index first
    int32_t iter, recounts, active, resample_pending;
    int32_t overflow, done, lower_pending, pad0;
    uint32_t tickets[4];
    unsigned long long lower_cnt[kMaxLower + 1];   // counts at t_1..t_m (multi-threshold pass)
};

struct SelWS {
    SelState* st;
    uint32_t* seg_cnt;
    uint32_t* seg_gt;
    uint32_t* seg_eq;
    uint16_t* lst_off;
    float* lst_val;
    unsigned long long* grp_cnt;   // zeroed region starts here ...
    unsigned long long* grp_gt;
    unsigned long long* grp_eq;    // ... ends here
    long long* grp_off;
    long long* grp_gt_off;
    long long* grp_eq_off;
    RSState* rs;
    int64_t nseg, ngrp;
    size_t zero_bytes;
};

static SelWS carve_select(void* base, int64_t numel, size_t* bytes = nullptr) {
    SelWS w{};
    w.nseg = ceil_div(numel, kSeg);
    w.ngrp = ceil_div(w.nseg, kGroupSegs);
    Carver c(base);
    w.st = c.take<SelState>(1);
    w.rs = c.take<RSState>(1);
    w.grp_cnt = c.take<unsigned long long>(3 * w.ngrp);
    w.grp_gt = w.grp_cnt ? w.grp_cnt + w.ngrp : nullptr;
    w.grp_eq = w.grp_gt ? w.grp_gt + w.ngrp : nullptr;
    w.zero_bytes = 3 * w.ngrp * sizeof(unsigned long long);
    w.grp_off = c.take<long long>(w.ngrp);
    w.grp_gt_off = c.take<long long>(w.ngrp);
    w.grp_eq_off = c.take<long long>(w.ngrp);
    w.seg_cnt = c.take<uint32_t>(w.nseg);
    w.seg_gt = c.take<uint32_t>(w.nseg);
    w.seg_eq = c.take<uint32_t>(w.nseg);
    w.lst_off = c.take<uint16_t>(w.nseg * kCap);
    w.lst_val = c.take<float>(w.nseg * kCap);
    if (bytes) *bytes = c.bytes();
    return w;
}

static size_t select_ws_bytes(int64_t numel) {
    size_t b = 0;
    carve_select(nullptr, numel, &b);
    return b;
}

// ------------------------------------------------------------------ tile loads
// Tile t of segment `seg`: lane holds elements e0..e0+3, e0 = seg*kSeg + t*256 + 4*lane.
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

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(kScanThreads) k_sel_init(SelWS w, const float* thr0) {
    SelState* st = w.st;
    for (int64_t i = threadIdx.x; i < 3 * w.ngrp; i += blockDim.x) w.grp_cnt[i] = 0;
    if (threadIdx.x == 0) {
        const float t = *thr0;
        st->t0 = t;
        st->t_cur = t;
        st->tk = 0.f;
        st->branch = -1;
        st->n_cur = st->limit = st->n_greater = st->tie_quota = 0;
        st->iter = st->recounts = 0;
        st->active = 1;
        st->resample_pending = 0;
        st->overflow = 0;
        st->done = 0;
        st->lower_pending = 0;
        for (int i = 0; i < 4; ++i) st->tickets[i] = 0;
        for (int i = 0; i <= kMaxLower; ++i) st->lower_cnt[i] = 0;
    }
}

// Select pass at st->t_cur: per-segment candidate lists + exact counts.
template <bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
k_select_pass(const float* __restrict__ vec, int64_t n, SelWS w) {
    if (!w.st->active) return;
    const float t = w.st->t_cur;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint32_t wcnt[kSegPerBlock];
    __shared__ uint32_t wovf[kSegPerBlock];
    // launched one-shot (grid = nseg/4: each block one iteration) for the first pass,
    // grid-stride with a capped grid for the gated recount passes
    for (int64_t bi = blockIdx.x; bi * kSegPerBlock < w.nseg; bi += gridDim.x) {
        const int64_t seg = bi * kSegPerBlock + wave;
        uint32_t c = 0;
        if (seg < w.nseg) {
            const int64_t base = seg * kSeg;
            uint16_t* lo = w.lst_off + seg * kCap;
            float* lv = w.lst_val + seg * kCap;
#pragma unroll
            for (int half = 0; half < kTiles / kSelBatch; ++half) {
                float x[kSelBatch][4];
                uint32_t valid[kSelBatch];
#pragma unroll
                for (int u = 0; u < kSelBatch; ++u)
                    load_tile<ALIGNED>(vec, n, base + (half * kSelBatch + u) * 256 + 4 * lane, x[u], valid[u]);
#pragma unroll
                for (int u = 0; u < kSelBatch; ++u) {
                    const uint32_t p = ge_mask(x[u], valid[u], t);
                    if (__ballot(p != 0)) {
                        uint32_t lb, tot;
                        wave_prefix4(p, lb, tot);
                        uint32_t r = c + lb;
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            if (p & (1u << j)) {
                                if (r < kCap) {
                                    lo[r] = (uint16_t)((half * kSelBatch + u) * 256 + 4 * lane + j);
                                    lv[r] = x[u][j];
                                }
                                ++r;
                            }
                        }
                        c += tot;
                    }
                }
            }
            if (lane == 0) w.seg_cnt[seg] = c;
        }
        if (lane == 0) {
            wcnt[wave] = c;
            wovf[wave] = c > kCap;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t s = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
            const uint32_t o = wovf[0] + wovf[1] + wovf[2] + wovf[3];
            if (s) atomicAdd(&w.grp_cnt[(bi * kSegPerBlock) / kGroupSegs], (unsigned long long)s);
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
// step is a recount (select pass + decide), exactly like the reference.
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
                    st->resample_pending = 1;
                    reset_rs = 1;
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
// max_iters) and arms the list pass + decide at t_{j*}.
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
    for (int64_t seg = (int64_t)blockIdx.x * kSegPerBlock + wave; seg < w.nseg;
         seg += (int64_t)gridDim.x * kSegPerBlock) {
        for (int tile = 0; tile < kTiles; ++tile) {
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
    __shared__ uint32_t part[kSegPerBlock][kMaxLower + 1];
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
        st->active = 1;   // list pass + decide at t_{j*}
    }
}

// Candidate keys of the final threshold, for the resample radix select: the
// segment's list when complete, a re-read of vec (|x| >= t_cur) when it spilled.
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
            const uint32_t c = w.seg_cnt[seg];
            if (c <= (uint32_t)kCap) {
                for (uint32_t e = lane; e < c; e += 64) f(abs_key(w.lst_val[seg * kCap + e]));
            } else {
                for (int tile = 0; tile < kTiles; ++tile) {
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

// Per-segment counts of |x| > tk and |x| == tk among the candidates (resample);
// the last workgroup scans the group totals and sets the tie quota k - #greater.
__global__ void __launch_bounds__(kBlock)
k_count_gt_eq(const float* __restrict__ vec, int64_t n, SelWS w, int64_t k) {
    SelState* st = w.st;
    if (!st->resample_pending) return;
    const float tk = st->tk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t bi = blockIdx.x; bi * kSegPerBlock < w.nseg; bi += gridDim.x) {
        const int64_t seg = bi * kSegPerBlock + wave;
        if (seg >= w.nseg) continue;
        uint32_t gt = 0, eq = 0;
        const uint32_t c = w.seg_cnt[seg];
        if (c <= (uint32_t)kCap) {
            for (uint32_t e = lane; e < c; e += 64) {
                const float a = fabsf(w.lst_val[seg * kCap + e]);
                gt += a > tk;
                eq += a == tk;
            }
        } else {
            for (int tile = 0; tile < kTiles; ++tile) {
                float x[4];
                uint32_t valid;
                load_tile<false>(vec, n, seg * kSeg + tile * 256 + 4 * lane, x, valid);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float a = fabsf(x[j]);
                    const bool ok = (valid >> j) & 1u;
                    gt += ok && a > tk;
                    eq += ok && a == tk;
                }
            }
        }
        gt = wave_sum(gt);
        eq = wave_sum(eq);
        if (lane == 0) {
            w.seg_gt[seg] = gt;
            w.seg_eq[seg] = eq;
            const int64_t g = seg / kGroupSegs;
            if (gt) atomicAdd(&w.grp_gt[g], (unsigned long long)gt);
            if (eq) atomicAdd(&w.grp_eq[g], (unsigned long long)eq);
        }
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

struct EmitOut {
    float* vec;          // null: leave vec untouched (pure selection)
    float* mmt;          // null: no momentum masking
    void* values;
    void* indices;
    int32_t vdtype, idtype;
};

__device__ __forceinline__ void emit_one(const EmitOut& o, int64_t pos, int64_t gidx, float x) {
    store_value(o.values, pos, x, o.vdtype);
    store_index(o.indices, pos, gidx, o.idtype);
    // scattered 4-B writes, one per 128-B line: non-temporal (no L2 allocation)
    if (o.vec) __builtin_nontemporal_store(0.f, o.vec + gidx);
    if (o.mmt) __builtin_nontemporal_store(0.f, o.mmt + gidx);
}

// Block-wide exclusive scan of one u32 per thread over a 256-thread block.
__device__ __forceinline__ uint32_t block_exclusive_scan_256(uint32_t v, uint32_t* lds4) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    if (lane == 63) lds4[wid] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int q = 0; q < wid; ++q) base += lds4[q];
    __syncthreads();
    return base + incl - v;
}

// Wave-cooperative emit of one segment by re-reading vec (a spilled list).
// FIRSTK: positions base + rank for |x| >= t, kept while < limit.
__device__ void emit_reread_firstk(const float* __restrict__ vec_in, int64_t n, int64_t seg, long long base,
                                   long long limit, float t, const EmitOut& o) {
    const int lane = threadIdx.x & 63;
    uint32_t run = 0;
    for (int tile = 0; tile < kTiles; ++tile) {
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
    for (int tile = 0; tile < kTiles; ++tile) {
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

// One workgroup per group of 256 segments, ONE THREAD PER SEGMENT for complete
// lists (a few entries each: no serial per-wave walk over segments), then the
// group's spilled segments, if any, one wave each.
__global__ void __launch_bounds__(kBlock)
k_emit(const float* __restrict__ vec_in, int64_t n, SelWS w, EmitOut o) {
    const SelState* st = w.st;
    const int mode = st->branch == DGC_BRANCH_RESAMPLE ? MODE_RESAMPLE : MODE_FIRSTK;
    const int64_t g = blockIdx.x;
    const int64_t s0 = g * kGroupSegs;
    const int nsg = (int)((w.nseg - s0) < kGroupSegs ? (w.nseg - s0) : kGroupSegs);
    const int ts = threadIdx.x, wave = threadIdx.x >> 6;
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t off_a[kGroupSegs], off_b[kGroupSegs];
    __shared__ int spill[kGroupSegs];
    __shared__ int nspill;
    if (ts == 0) nspill = 0;
    const int64_t seg = s0 + ts;
    const uint32_t c = ts < nsg ? w.seg_cnt[seg] : 0;
    if (mode == MODE_FIRSTK) {
        off_a[ts] = block_exclusive_scan_256(c, lds4);
    } else {
        const uint32_t a = ts < nsg ? w.seg_gt[seg] : 0;
        const uint32_t b = ts < nsg ? w.seg_eq[seg] : 0;
        off_a[ts] = block_exclusive_scan_256(a, lds4);
        off_b[ts] = block_exclusive_scan_256(b, lds4);
    }
    __syncthreads();
    const uint16_t* lo = w.lst_off + seg * kCap;
    const float* lv = w.lst_val + seg * kCap;
    if (mode == MODE_FIRSTK) {
        const long long limit = st->limit;
        const long long base = w.grp_off[g] + off_a[ts];
        if (ts < nsg && c > 0 && base < limit) {
            if (c <= (uint32_t)kCap) {
                const long long m = (limit - base) < (long long)c ? (limit - base) : (long long)c;
                for (long long e = 0; e < m; ++e) emit_one(o, base + e, seg * kSeg + lo[e], lv[e]);
            } else {
                spill[atomicAdd(&nspill, 1)] = ts;
            }
        }
        __syncthreads();
        const float t = st->t_cur;
        for (int q = wave; q < nspill; q += kSegPerBlock) {
            const int sl = spill[q];
            emit_reread_firstk(vec_in, n, s0 + sl, w.grp_off[g] + off_a[sl], limit, t, o);
        }
    } else {
        const float tk = st->tk;
        const long long T = st->tie_quota;
        if (ts < nsg && c > 0) {
            const long long bg = w.grp_gt_off[g] + off_a[ts];
            const long long bt = w.grp_eq_off[g] + off_b[ts];
            if (c <= (uint32_t)kCap) {
                long long rg = 0, rt = 0;
                for (uint32_t e = 0; e < c; ++e) {
                    const float x = lv[e];
                    const float a = fabsf(x);
                    const bool gt = a > tk, eq = a == tk;
                    const long long tb = bt + rt;
                    if (gt || (eq && tb < T)) emit_one(o, bg + rg + (tb < T ? tb : T), seg * kSeg + lo[e], x);
                    rg += gt;
                    rt += eq;
                }
            } else {
                spill[atomicAdd(&nspill, 1)] = ts;
            }
        }
        __syncthreads();
        for (int q = wave; q < nspill; q += kSegPerBlock) {
            const int sl = spill[q];
            emit_reread_resample(vec_in, n, s0 + sl, w.grp_gt_off[g] + off_a[sl], w.grp_eq_off[g] + off_b[sl], tk,
                                 T, o);
        }
    }
}

__global__ void k_sel_finish(const SelState* st, int64_t k, int64_t* count_out, dgc_select_info* info) {
    if (threadIdx.x != 0) return;
    const long long cnt = st->branch == DGC_BRANCH_RESAMPLE ? k : st->limit;
    if (count_out) *count_out = cnt;
    if (info) {
        info->count = cnt;
        info->candidates = st->n_cur;
        info->threshold0 = st->t0;
        info->threshold = st->t_cur;
        info->branch = st->branch;
        info->recounts = st->recounts;
        info->overflow_segments = st->overflow;
        info->reserved = 0;
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

int select(float* vec, float* mmt, const float* thr0, const dgc_select_params* p, void* values,
           void* indices, int64_t* count_out, dgc_select_info* info, void* ws, size_t ws_bytes,
           int sync_mode, hipStream_t s) {
    DGC_TRY(validate_select(p, values, indices));
    if (!vec || !thr0 || (p->update_memory && p->masking && !mmt))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null vec/thr0/mmt");
    const int64_t n = p->numel;
    if (!ws || ws_bytes < select_ws_bytes(n) || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_select: workspace needs %zu bytes, 256-B aligned",
                 select_ws_bytes(n));
    SelWS w = carve_select(ws, n);
    hipLaunchKernelGGL(k_sel_init, dim3(1), dim3(kScanThreads), 0, s, w, thr0);
    DGC_LAUNCHED();
    const int grid = (int)ceil_div(w.nseg, kSegPerBlock);      // one-shot select-pass blocks
    const int grid_gs = grid_for(w.nseg, kSegPerBlock);         // grid-stride (gated) kernels
    const bool al = aligned16(vec);
    const bool adapt = p->numel > p->num_samples;
    const bool lower_fast = p->resample && p->max_iters <= kMaxLower;
    auto pass = [&](int blocks) -> int {
        if (al)
            hipLaunchKernelGGL(k_select_pass<true>, dim3(blocks), dim3(kBlock), 0, s, vec, n, w);
        else
            hipLaunchKernelGGL(k_select_pass<false>, dim3(blocks), dim3(kBlock), 0, s, vec, n, w);
        DGC_LAUNCHED();
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
    auto resample = [&]() -> int {
        // rs state reset by k_decide when it chose the resample branch
        CandKeys src{vec, n, w};
        DGC_TRY(radix_select_passes(src, grid_gs, &w.st->tk, w.rs, &w.st->resample_pending, s));
        hipLaunchKernelGGL(k_count_gt_eq, dim3(grid_gs), dim3(kBlock), 0, s, vec, n, w, (int64_t)p->num_selects);
        DGC_LAUNCHED();
        return DGC_OK;
    };
    DGC_TRY(pass(grid));
    if (sync_mode == DGC_SYNC_HOST) {
        // read each decision back and launch only what it needs
        SelState hs{};
        for (;;) {
            DGC_HIP(hipMemcpyAsync(&hs, w.st, sizeof(hs), hipMemcpyDeviceToHost, s));
            DGC_HIP(hipStreamSynchronize(s));
            if (hs.done) break;
            if (hs.lower_pending) DGC_TRY(lower());
            DGC_TRY(pass(grid));
        }
        if (hs.branch == DGC_BRANCH_RESAMPLE) DGC_TRY(resample());
    } else if (adapt) {
        // every kernel below early-exits on a device flag when it is not needed
        if (lower_fast) {
            DGC_TRY(lower());
            DGC_TRY(pass(grid_gs));
        } else {
            for (int i = 0; i < p->max_iters; ++i) DGC_TRY(pass(grid_gs));
        }
        if (p->resample) DGC_TRY(resample());
    }
    EmitOut o{p->update_memory ? vec : nullptr, (p->update_memory && p->masking) ? mmt : nullptr, values,
              indices, p->vdtype, p->idtype};
    hipLaunchKernelGGL(k_emit, dim3((unsigned)w.ngrp), dim3(kBlock), 0, s, vec, n, w, o);
    DGC_LAUNCHED();
    hipLaunchKernelGGL(k_sel_finish, dim3(1), dim3(64), 0, s, w.st, (int64_t)p->num_selects,
                       count_out, info);
    DGC_LAUNCHED();
    return DGC_OK;
}

// ------------------------------------------------------------------ threshold
static size_t kth_ws_bytes(int64_t n) { return n <= kSmallN ? 256 : align_up(sizeof(RSState), 256); }

int kth_largest(const float* x, int64_t n, int64_t k, float* out, void* ws, size_t ws_bytes,
                hipStream_t s) {
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

struct CompressWS {
    float* thr;
    float* samples;
    RSState* rs;
    void* sel;
    size_t sel_bytes;
};

// sample_buf: floats reserved for the strided samples (0 when numel == num_samples)
static CompressWS carve_compress(void* base, int64_t numel, int64_t sample_buf, size_t* bytes = nullptr) {
    Carver c(base);
    CompressWS w{};
    w.thr = c.take<float>(64);
    w.rs = c.take<RSState>(1);
    w.samples = c.take<float>(sample_buf);
    w.sel_bytes = select_ws_bytes(numel);
    w.sel = c.take<char>(w.sel_bytes);
    if (bytes) *bytes = c.bytes();
    return w;
}

static size_t compress_ws_bytes(int64_t numel, int64_t sample_buf) {
    size_t b = 0;
    carve_compress(nullptr, numel, sample_buf, &b);
    return b;
}

int compress(const float* grad, float* mmt, float* vec, float momentum, bool nesterov,
             int64_t s_start, int64_t s_stride, int64_t top_k_samples, const dgc_select_params* p,
             void* values, void* indices, int64_t* count_out, dgc_select_info* info, void* ws,
             size_t ws_bytes, int sync_mode, hipStream_t s) {
    DGC_TRY(validate_select(p, values, indices));
    const int64_t n = p->numel;
    const bool sampled = n != p->num_samples;
    const int64_t L = sampled ? ceil_div(n - s_start, s_stride) : n;
    if (sampled && (s_stride < 2 || s_start < 0 || s_start >= s_stride))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: sample_start must be in [0, stride)");
    if (top_k_samples < 1 || top_k_samples > L)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: top_k_samples %lld outside [1, %lld]",
                 (long long)top_k_samples, (long long)L);
    const int64_t sbuf = sampled ? L : 0;
    if (!ws || ws_bytes < compress_ws_bytes(n, sbuf) || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_compress: workspace needs %zu bytes, 256-B aligned",
                 compress_ws_bytes(n, sbuf));
    CompressWS w = carve_compress(ws, n, sbuf);
    // K1 (+ fused strided sample of |vec|)
    DGC_TRY(compensate(grad, mmt, vec, nullptr, n, momentum, nesterov, true, sampled ? w.samples : nullptr,
                       s_start, s_stride, sampled ? L : 0, s));
    // K3: threshold = k-th largest sample (|vec| itself when numel == num_samples)
    const float* src = sampled ? w.samples : vec;
    DGC_TRY(kth_largest(src, L, top_k_samples, w.thr, w.rs, sizeof(RSState), s));
    // K4 (+ DGCSGDMemory.update fused into the emit)
    dgc_select_params q = *p;
    q.update_memory = 1;
    return select(vec, mmt, w.thr, &q, values, indices, count_out, info, w.sel, w.sel_bytes, sync_mode, s);
}

}  // namespace dgc

// ------------------------------------------------------------------ C ABI
extern "C" size_t dgc_kth_largest_workspace(int64_t n) { return dgc::kth_ws_bytes(n); }

extern "C" int dgc_kth_largest(const float* x, int64_t n, int64_t k, float* thr_out, void* ws,
                               size_t ws_bytes, void* stream) {
    return dgc::kth_largest(x, n, k, thr_out, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" size_t dgc_select_workspace(int64_t numel, int64_t num_selects) {
    (void)num_selects;
    return dgc::select_ws_bytes(numel);
}

extern "C" int dgc_select(float* vec, float* mmt, const float* thr0, const dgc_select_params* params,
                          void* values_out, void* indices_out, int64_t* count_out,
                          dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                          void* stream) {
    return dgc::select(vec, mmt, thr0, params, values_out, indices_out, count_out, info_out, ws, ws_bytes,
                       sync_mode, static_cast<hipStream_t>(stream));
}

extern "C" size_t dgc_compress_workspace(int64_t numel, int64_t num_selects, int64_t num_samples) {
    (void)num_selects;
    // the strided slice holds ceil((numel - start) / stride) <= num_samples + 1 samples
    return dgc::compress_ws_bytes(numel, numel == num_samples ? 0 : num_samples + 1);
}

extern "C" int dgc_compress(const float* grad, float* mmt, float* vec, float momentum, int32_t nesterov,
                            int64_t sample_start, int64_t sample_stride, int64_t top_k_samples,
                            const dgc_select_params* params, void* values_out, void* indices_out,
                            int64_t* count_out, dgc_select_info* info_out, void* ws, size_t ws_bytes,
                            int32_t sync_mode, void* stream) {
    return dgc::compress(grad, mmt, vec, momentum, nesterov != 0, sample_start, sample_stride,
                         top_k_samples, params, values_out, indices_out, count_out, info_out, ws,
                         ws_bytes, sync_mode, static_cast<hipStream_t>(stream));
}
