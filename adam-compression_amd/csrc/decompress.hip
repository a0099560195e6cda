// K6: deterministic decompress = grad.zero_().index_put_([idx], vals, accumulate=True)
// followed by grad.mul_(1/W) (dgc/compression.py:179-194), over the rank-order
// concatenation that the allgather produced (dgc/compression.py:200-212).
//
// The reference's single-threaded CPU index_put_ adds entries in input order. The
// input is a sequence of RUNS (one per rank; our compress emits each rank's indices
// ascending), so the dense result is reproduced bit-for-bit without atomics:
//
//   zero    dgc_fill_zero: one-shot 16-B stores over grad (the reference's zero_());
//   bounds  one coalesced pass over every run's entries marks, per (run, 4096-element
//           chunk), the first entry whose index reaches the chunk;
//   scatter one run: a thread per entry. Several runs: a wave per super-chunk of
//           ~32 entries, lane order = rank order; an index seen in two runs (an LDS
//           bitmap finds it) is summed in lane order by its first occurrence, so
//           every sum has the sequential order; then * (1/W) and one 4-B store per
//           index. Crowded super-chunks go to a workgroup path that accumulates in
//           registers in the same order.
//
// HBM: the dense write (4 B/elem) plus the sparse reads W*k*(vb+ib) and one
// scattered store per distinct index. Untouched slots come out +0.0 exactly as
// zero_() * (1/W).
#include "dgc_common.hpp"

#include <mutex>
#include <utility>
#include <vector>

namespace dgc {

constexpr int kChunk = 4096;
constexpr int kMaxRuns = 64;
constexpr int kSegWaves = kBlock / kWave;   // waves per workgroup

struct Run {
    const void* vals;
    const void* idx;
    long long count;
};

struct DecWS {
    Run* runs;
    int32_t* nruns;
    int32_t* status;      // bit 0: index out of range, bit 1: a run out of order, bit 2: a header count
                          // outside [0, capacity] (that run is clamped)
    int32_t* sink;        // null, or the host-mapped words [index, count] bound to this workspace
                          // (dgc_decompress_bind_sink): the error bits also land there
    int32_t* ndesc;       // detected descents
    int32_t* ovf_cnt;     // sparse scatter: super-chunks queued for the workgroup path
    int32_t* ovf_list;
    long long* desc;      // their positions (unsorted)
    long long* bnd;       // [kMaxRuns][nchunks + 1]
    int64_t nchunks;
    // runs that are not non-decreasing (a resample payload in the reference's topk
    // order) are regrouped by chunk before the scatter: flag, regrouped run, cursors,
    // and a copy area of sort_cap entries per run (0: no regrouping, the flag only)
    int32_t* unsorted;    // [kMaxRuns]
    Run* sorted;          // [kMaxRuns]
    uint32_t* cursor;     // [max_runs][nchunks]
    char* sort_buf;       // [max_runs][sort_cap * 12 B]
    int64_t sort_cap;
};

int32_t* bound_sink(const void* ws);

static DecWS carve_dec(void* base, int64_t n, int32_t max_runs, int64_t sort_cap = 0, size_t* bytes = nullptr) {
    Carver c(base);
    DecWS w{};
    w.sink = base ? bound_sink(base) : nullptr;
    w.nchunks = ceil_div(n, kChunk);
    w.runs = c.take<Run>(kMaxRuns);
    w.nruns = c.take<int32_t>(4);
    w.status = w.nruns ? w.nruns + 1 : nullptr;
    w.ndesc = w.nruns ? w.nruns + 2 : nullptr;
    w.ovf_cnt = w.nruns ? w.nruns + 3 : nullptr;
    w.desc = c.take<long long>(kMaxRuns);
    w.bnd = c.take<long long>((size_t)max_runs * (w.nchunks + 1));
    w.ovf_list = c.take<int32_t>(w.nchunks);
    w.unsorted = c.take<int32_t>(kMaxRuns);
    w.sorted = c.take<Run>(kMaxRuns);
    w.sort_cap = sort_cap;
    w.cursor = c.take<uint32_t>(sort_cap ? (size_t)max_runs * w.nchunks : 0);
    w.sort_buf = c.take<char>(sort_cap ? (size_t)max_runs * sort_cap * 12 : 0);
    if (bytes) *bytes = c.bytes();
    return w;
}

// An index outside [0, n) (dropped from the sum; the reference's index_put_ raises), or
// a gathered header count outside [0, capacity] (the run is clamped): the status word
// for dgc_decompress_status, and the bound sink for an engine's per-step check.
__device__ __forceinline__ void flag_index(const DecWS& w) {
    atomicOr(w.status, 1);
    raise_flag(w.sink);
}
__device__ __forceinline__ void flag_count(const DecWS& w) {
    atomicOr(w.status, 4);
    raise_flag(w.sink ? w.sink + 1 : nullptr);
}

template <int VD>
__device__ __forceinline__ float load_val(const void* p, long long e) {
    if (VD == DGC_F16) return (float)((const DGC_GLB _Float16*)p)[e];   // typed: global_ loads; exact widening
    return ((const DGC_GLB float*)p)[e];
}

template <int ID>
__device__ __forceinline__ long long load_idx(const void* p, long long e) {
    if (ID == DGC_I32) return ((const DGC_GLB int32_t*)p)[e];
    return ((const DGC_GLB int64_t*)p)[e];
}

// Where the runs come from: a table in the workspace (concatenated input), or the
// packed allgather buffer itself (rank r's header holds its count) — the latter
// needs no setup launch. A split exchange (dgc_payload_split) gathers each rank's
// payload as `parts` part buffers, part-major (part p of rank r at p * pstride +
// r * stride): run q = r * parts + p, so the runs stay in rank order (an index is in
// at most one part of a rank); parts >= `ready` have not landed yet and are empty.
struct RunSrc {
    const Run* table;
    const int32_t* nruns_dev;
    const char* payload;          // packed mode when non-null
    int64_t stride, voff, ioff, capacity;
    int32_t world;
    const int32_t* unsorted;      // regrouped runs (null: none): read them from `sorted`
    const Run* sorted;
    int32_t parts = 1, ready = 1;
    int64_t pstride = 0;
    __host__ __device__ __forceinline__ int count() const { return payload ? world * parts : *nruns_dev; }
    __device__ __forceinline__ Run get(int r) const {
        if (unsorted && unsorted[r]) return sorted[r];
        return get_raw(r);
    }
    __device__ __forceinline__ const char* base_of(int q) const {
        const int r = q / parts, p = q - r * parts;
        return payload + (int64_t)p * pstride + (int64_t)r * stride;
    }
    // the header's count as gathered (packed mode, a part that has landed), unclamped
    __device__ __forceinline__ long long raw_count(int q) const {
        if (!payload || (parts > 1 && q % parts >= ready)) return 0;
        return *reinterpret_cast<const long long*>(base_of(q));
    }
    __device__ __forceinline__ Run get_raw(int q) const {
        if (!payload) return table[q];
        const char* base = base_of(q);
        if (parts > 1 && q % parts >= ready) return Run{base + voff, base + ioff, 0};
        long long c = *reinterpret_cast<const long long*>(base);
        c = c < 0 ? 0 : (c > capacity ? capacity : c);
        return Run{base + voff, base + ioff, c};
    }
    // split exchange: min over ranks of the smallest index in the parts after part p
    // (header word 1, dgc_payload_split); every index below it has landed with parts <= p
    __device__ __forceinline__ long long landed_below(int p) const {
        long long m = LLONG_MAX;
        for (int r = 0; r < world; ++r) {
            const long long b = reinterpret_cast<const long long*>(base_of(r * parts + p))[1];
            m = b < m ? b : m;
        }
        return m;
    }
};

// ---------------------------------------------------------------- run tables
struct HostRuns {
    int32_t n;
    long long off[kMaxRuns + 1];
};

__global__ void k_runs_host(DecWS w, HostRuns hr, const char* vals, const char* idx, int vb, int ib) {
    const int r = threadIdx.x;
    if (r < hr.n) w.runs[r] = Run{vals + hr.off[r] * vb, idx + hr.off[r] * ib, hr.off[r + 1] - hr.off[r]};
    if (r == 0) *w.nruns = hr.n;
}

template <int ID>
__global__ void __launch_bounds__(kBlock)
k_find_descents(const void* idx, long long total, DecWS w) {
    for (long long j = (long long)blockIdx.x * kBlock + threadIdx.x; j + 1 < total;
         j += (long long)gridDim.x * kBlock) {
        if (load_idx<ID>(idx, j + 1) < load_idx<ID>(idx, j)) {
            const int slot = atomicAdd(w.ndesc, 1);
            if (slot < kMaxRuns - 1) w.desc[slot] = j + 1;
        }
    }
}

__global__ void k_runs_from_descents(DecWS w, const char* vals, const char* idx, int vb, int ib,
                                     long long total) {
    if (threadIdx.x != 0) return;
    int nd = *w.ndesc;
    if (nd > kMaxRuns - 1) {
        *w.nruns = 0;
        return;
    }
    long long* d = w.desc;
    for (int i = 1; i < nd; ++i) {   // insertion sort, <= 63 entries
        const long long v = d[i];
        int j = i - 1;
        while (j >= 0 && d[j] > v) {
            d[j + 1] = d[j];
            --j;
        }
        d[j + 1] = v;
    }
    long long prev = 0;
    for (int r = 0; r <= nd; ++r) {
        const long long end = r < nd ? d[r] : total;
        w.runs[r] = Run{vals + prev * vb, idx + prev * ib, end - prev};
        prev = end;
    }
    *w.nruns = nd + 1;
}

// ---------------------------------------------------------------- bounds
// bnd[r][c] = the first entry of run r whose index reaches key_c (key_c = 4096c for
// c < nchunks, key_nchunks = n), i.e. what a binary search per (run, chunk) would
// give — built instead from one coalesced pass over the entries. With
// G(v) = #{c : key_c <= v}, entry e owns the chunks c in [G(idx[e-1]), G(idx[e]))
// (G(idx[-1]) = 0, G(idx[count]) = nchunks + 1), so every bnd slot is written once
// by the entry that starts it. Ranges longer than 8 chunks (gaps, empty runs) are
// written by the whole wave. A descending pair (an unsorted run) sets status bit 2;
// such a run can leave slots unwritten, so readers clamp bnd to [0, count].
__device__ __forceinline__ long long chunk_rank(long long v, int64_t n, int64_t nchunks) {
    if (v < 0) return 0;
    const long long c = (v >> 12) < nchunks - 1 ? (v >> 12) : nchunks - 1;
    return c + 1 + (v >= n ? 1 : 0);
}

template <int ID>
__global__ void __launch_bounds__(kBlock)
k_bounds(DecWS w, RunSrc rs, int64_t n, int64_t cap, int ystep, int yoff) {
    const int r = (int)blockIdx.y * ystep + yoff;   // the run (a split exchange: one part's runs)
    const int64_t stride = w.nchunks + 1;
    if (r >= rs.count()) return;   // uniform per workgroup
    const Run run = rs.get_raw(r);
    long long* bnd = w.bnd + (int64_t)r * stride;
    const int lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const long long c = rs.raw_count(r);
        if (c < 0 || c > rs.capacity) flag_count(w);
    }
    for (int64_t e0 = (int64_t)blockIdx.x * kBlock; e0 <= run.count; e0 += (int64_t)gridDim.x * kBlock) {
        const int64_t e = e0 + threadIdx.x;
        long long lo = 0, hi = 0;
        if (e <= run.count) {
            const long long ip = e > 0 ? load_idx<ID>(run.idx, e - 1) : -1;
            const long long ic = e < run.count ? load_idx<ID>(run.idx, e) : 0;
            lo = e > 0 ? chunk_rank(ip, n, w.nchunks) : 0;
            hi = e < run.count ? chunk_rank(ic, n, w.nchunks) : stride;
            if (e < run.count && (ic < 0 || ic >= n)) flag_index(w);
            if (e > 0 && e < run.count && ic < ip) {
                atomicOr(w.status, 2);
                if (w.sort_cap) atomicOr(&w.unsorted[r], 1);
            }
            if (hi < lo) hi = lo;
        }
        if (hi - lo <= 8) {
            for (long long c = lo; c < hi; ++c) bnd[c] = e;
        }
        uint64_t longs = __ballot(hi - lo > 8);
        while (longs) {
            const int L = __builtin_ctzll(longs);
            longs &= longs - 1;
            const long long a = __shfl(lo, L), b = __shfl(hi, L);
            const long long v = e0 + (threadIdx.x & ~63) + L;
            for (long long c = a + lane; c < b; c += 64) bnd[c] = v;
        }
    }
}

// Entries [b0, b1) of run r for chunk c, clamped so stale bounds (unsorted runs) stay in range.
__device__ __forceinline__ void chunk_range(const long long* bnd, int64_t c, long long count, long long& b0,
                                            long long& b1) {
    b0 = bnd[c];
    b1 = bnd[c + 1];
    b0 = b0 < 0 ? 0 : (b0 > count ? count : b0);
    b1 = b1 < b0 ? b0 : (b1 > count ? count : b1);
}

// ---------------------------------------------------------------- unsorted runs
// A run k_bounds found out of order — the reference's resample sends its indices in
// torch.topk's order (dgc/compression.py:134-137) — is regrouped by chunk, one
// workgroup per run: counts per chunk, scan (= its bnd row), then every entry is
// copied to its chunk's next slot. Within a chunk the copy's order is arbitrary;
// indices are unique within a run (every DGC payload), so each index still gets one
// term per run and the scatter keeps the rank order of the terms: the sums are the
// sequential index_put_ sums.
constexpr int kRegroupThreads = 1024;

template <int VD, int ID>
__global__ void __launch_bounds__(kRegroupThreads) k_regroup(DecWS w, RunSrc rs, int64_t n, int ystep, int yoff) {
    const int r = (int)blockIdx.x * ystep + yoff;
    if (r >= rs.count() || !w.unsorted[r]) return;   // uniform per workgroup
    const Run run = rs.get_raw(r);
    const int64_t stride = w.nchunks + 1;
    long long* bnd = w.bnd + (int64_t)r * stride;
    uint32_t* cur = w.cursor + (int64_t)r * w.nchunks;
    const int tid = threadIdx.x;
    for (int64_t c = tid; c < stride; c += kRegroupThreads) bnd[c] = 0;
    __syncthreads();
    for (long long e = tid; e < run.count; e += kRegroupThreads) {
        const long long i = load_idx<ID>(run.idx, e);
        if (i < 0 || i >= n) {
            flag_index(w);
            continue;
        }
        atomicAdd((unsigned long long*)&bnd[(i >> 12) + 1], 1ull);
    }
    __syncthreads();
    // inclusive scan of bnd[0..stride): bnd[c] = first slot of chunk c, bnd[nchunks] = in-range entries
    __shared__ uint64_t lds16[16];
    const int64_t per = ceil_div(stride, (int64_t)kRegroupThreads);
    const int64_t b = tid * per, e = b + per < stride ? b + per : stride;
    uint64_t local = 0;
    for (int64_t c = b; c < e; ++c) local += (uint64_t)bnd[c];
    uint64_t total;
    uint64_t run_sum = block_exclusive_scan(local, lds16, &total);
    for (int64_t c = b; c < e; ++c) {
        run_sum += (uint64_t)bnd[c];
        bnd[c] = (long long)run_sum;
        if (c < w.nchunks) cur[c] = (uint32_t)run_sum;
    }
    __syncthreads();
    char* base = w.sort_buf + (int64_t)r * w.sort_cap * 12;
    void* sv = base;
    void* si = base + w.sort_cap * 4;
    for (long long e2 = tid; e2 < run.count; e2 += kRegroupThreads) {
        const long long i = load_idx<ID>(run.idx, e2);
        if (i < 0 || i >= n) continue;
        const uint32_t pos = atomicAdd(&cur[i >> 12], 1u);
        if (VD == DGC_F16)
            reinterpret_cast<__half*>(sv)[pos] = reinterpret_cast<const __half*>(run.vals)[e2];
        else
            reinterpret_cast<float*>(sv)[pos] = reinterpret_cast<const float*>(run.vals)[e2];
        if (ID == DGC_I32)
            reinterpret_cast<int32_t*>(si)[pos] = (int32_t)i;
        else
            reinterpret_cast<int64_t*>(si)[pos] = i;
    }
    if (tid == 0) w.sorted[r] = Run{sv, si, (long long)bnd[w.nchunks]};
}

// ---------------------------------------------------------------- crowded chunks
// One 4096-element chunk per workgroup, for chunks too crowded for one wave (see
// k_scatter_waves); grad already holds +0.0 there. Thread t owns the float4s t,
// t+256, t+512, t+768 of the chunk in registers, starting at +0.0. The chunk's
// entries are staged in LDS in RUN ORDER (batches of kTileStage) and every wave walks
// them in that order, adding each entry it owns into the owning lane's register —
// the sequential index_put_ order (repeats included), so sums are bit-exact with no
// atomics. Then * (1/W), and the touched elements are stored.
constexpr int kTileStage = 1024;

template <int VD, int ID>
__device__ void tile_chunk(const DecWS& w, const RunSrc& rs, float* __restrict__ grad, int64_t n, float scale,
                           int64_t c) {
    __shared__ int soff[kTileStage];
    __shared__ float sval[kTileStage];
    __shared__ int roff[kMaxRuns + 1];
    __shared__ long long rb0[kMaxRuns];
    __shared__ const void* rval[kMaxRuns];
    __shared__ const void* ridx[kMaxRuns];
    const int nr = rs.count();
    const int64_t stride = w.nchunks + 1;
    const long long base = c * (long long)kChunk;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 64) {   // run table of this chunk (nr <= 64: one wave)
        long long cnt = 0;
        if (tid < nr) {
            const Run run = rs.get(tid);
            const long long* bnd = w.bnd + (int64_t)tid * stride;
            long long b0, b1;
            chunk_range(bnd, c, run.count, b0, b1);
            rb0[tid] = b0;
            rval[tid] = run.vals;
            ridx[tid] = run.idx;
            cnt = b1 - b0;
            // idx < 0 or >= n; a split phase's runs that have not landed (count 0) have no
            // bounds yet (their slots hold an earlier call's)
            if (c == 0 && run.count > 0 && (bnd[0] > 0 || bnd[w.nchunks] < run.count)) flag_index(w);
        }
        const long long incl = (long long)wave_incl_scan64((uint64_t)cnt);   // the whole wave 0 is here
        if (tid < nr) roff[tid] = (int)(incl - cnt);
        if (tid == nr - 1) roff[nr] = (int)incl;
    }
    __syncthreads();
    const int total = roff[nr];
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = 0.f;
    uint32_t touched = 0;
    for (int t0 = 0; t0 < total; t0 += kTileStage) {
        const int m = total - t0 < kTileStage ? total - t0 : kTileStage;
        for (int t = tid; t < m; t += kBlock) {
            int r = 0;
            while (roff[r + 1] <= t0 + t) ++r;   // <= 64 runs
            const long long e = rb0[r] + (t0 + t - roff[r]);
            const long long off = load_idx<ID>(ridx[r], e) - base;
            soff[t] = (off >= 0 && off < kChunk) ? (int)off : -1;
            sval[t] = load_val<VD>(rval[r], e);
        }
        __syncthreads();
        for (int t = 0; t < m; ++t) {
            const int off = __builtin_amdgcn_readfirstlane(soff[t]);   // uniform: scalar branches
            if (off < 0) {
                if (tid == 0) atomicOr(w.status, 2);   // only an unsorted run lands outside its chunk
                continue;
            }
            if (((off >> 8) & 3) != wave) continue;
            const float v = sval[t];
            if (((off >> 2) & 63) == lane) {
                const int slot = ((off >> 10) << 2) | (off & 3);
                touched |= 1u << slot;
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (j == slot) a[j] = __fadd_rn(a[j], v);
            }
        }
        __syncthreads();
    }
    if (scale != 1.0f) {
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = __fmul_rn(a[j], scale);
    }
    if (!touched) return;
    const long long len = n - base < kChunk ? n - base : kChunk;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const long long e = (long long)(u * kBlock + tid) * 4 + j;
            if (e < len && ((touched >> (4 * u + j)) & 1u)) grad[base + e] = a[4 * u + j];
        }
}

// ---------------------------------------------------------------- sparse scatter
// grad holds +0.0 on entry (the reference's zero_(), done earlier); only the entries
// are written. The work scales with the entries, not with n.
//
// One run (W = 1): four threads per entry. The first of a repeat sums the repeats in
// order (index_put_ order); a descent or an index outside [0, n) sets the status.
// An engine payload whose indices ascend (header word 1 = DGC_ORDER_ASCENDING, written
// by the selection's finish) has each 64-B granule's entries next to each other, so
// the first entry of a granule writes the WHOLE granule — its entries' sums, +0.0
// around them (what grad holds there) — one 16-B quarter per thread: full-granule
// stores instead of 4-B partial writes (1.7x the line rate at scattered lines,
// tools/scatterbench.hip). Otherwise (the exact replays' topk order, run tables) the
// first thread of each entry stores its word.
template <int VD, int ID>
__global__ void __launch_bounds__(kBlock)
k_scatter_single(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale) {
    const Run run = rs.get_raw(0);   // any order: one run's unique indices need no regrouping
    const bool gran = rs.payload != nullptr &&
                      reinterpret_cast<const long long*>(rs.base_of(0))[1] == (long long)DGC_ORDER_ASCENDING;
    const long long t = (long long)blockIdx.x * kBlock + threadIdx.x;
    const long long j = t >> 2;
    const int part = (int)(t & 3);
    if (t == 0) {
        const long long c = rs.raw_count(0);
        if (c < 0 || c > rs.capacity) flag_count(w);
    }
    if (j >= run.count) return;
    const long long i = load_idx<ID>(run.idx, j);
    const long long ip = j > 0 ? load_idx<ID>(run.idx, j - 1) : -1;
    if (part == 0 && j > 0 && ip > i) atomicOr(w.status, 2);
    if (i < 0 || i >= n) {
        if (part == 0) flag_index(w);
        return;
    }
    const uintptr_t lo = reinterpret_cast<uintptr_t>(grad), hi = reinterpret_cast<uintptr_t>(grad + n);
    const uintptr_t g = reinterpret_cast<uintptr_t>(grad + i) & ~(uintptr_t)63;
    if (gran && g >= lo && g + 64 <= hi) {
        // the granule's first entry only (a predecessor in the same granule -> not first)
        if (j > 0 && ip >= 0 && (reinterpret_cast<uintptr_t>(grad + ip) & ~(uintptr_t)63) == g) return;
        const long long e0 = (long long)((g - lo) >> 2) + 4 * part;   // this thread's 4 elements
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        bool any[4] = {false, false, false, false};
        for (long long f = j; f < run.count; ++f) {
            const long long x = f == j ? i : load_idx<ID>(run.idx, f);
            if (x < 0 || x >= n || (reinterpret_cast<uintptr_t>(grad + x) & ~(uintptr_t)63) != g) break;
            const long long q = x - e0;
            if (q >= 0 && q < 4) {
                const float v = load_val<VD>(run.vals, f);
                a[q] = any[q] ? __fadd_rn(a[q], v) : __fadd_rn(0.f, v);
                any[q] = true;
            }
        }
        if (scale != 1.0f)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (any[q]) a[q] = __fmul_rn(a[q], scale);
        reinterpret_cast<DGC_GLB f4v*>(g)[part] = f4v{a[0], a[1], a[2], a[3]};
        return;
    }
    if (part != 0 || (j > 0 && ip == i)) return;   // one word per distinct index, by its first entry
    float a = __fadd_rn(0.f, load_val<VD>(run.vals, j));
    for (long long f = j + 1; f < run.count && load_idx<ID>(run.idx, f) == i; ++f)
        a = __fadd_rn(a, load_val<VD>(run.vals, f));
    grad[i] = scale != 1.0f ? __fmul_rn(a, scale) : a;
}

// Several runs: one wave per kSCB super-chunks of m 4096-element chunks each, m
// chosen on the host so a super-chunk holds ~32 entries. Every load the wave needs is
// issued up front for all kSCB super-chunks (the run bounds, then the entries), so a
// wave waits for two memory round trips per kSCB super-chunks, not per super-chunk.
// Inside a super-chunk, lane l takes entry l (runs concatenated in rank order, so
// lane order IS the index_put_ order); the lane holding the first occurrence of an
// index sums every occurrence in lane order through wave shuffles. A super-chunk
// with more than 64 entries is queued for the workgroup path (tile_chunk per
// 4096-element chunk, a second kernel).
constexpr int kSCB = 4;
constexpr int kGranules = 256;   // per-wave granule counters (a power of two)

// LDS writes of this wave visible to its later LDS reads (wave-synchronous code).
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int VD, int ID>
__global__ void __launch_bounds__(kBlock)
k_scatter_waves(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale, int m, int gran) {
    // per-wave duplicate filter: one bit per (offset mod 4096) of the super-chunk; and
    // per-granule counts of the entries to store (64-B granule, mod kGranules)
    __shared__ uint32_t dup_bits[kSegWaves][kChunk / 32];
    __shared__ uint32_t gran_cnt[kSegWaves][kGranules];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* bits = dup_bits[wv];
    uint32_t* gcnt = gran_cnt[wv];
    for (int q = lane; q < kChunk / 32; q += 64) bits[q] = 0;
    for (int q = lane; q < kGranules; q += 64) gcnt[q] = 0;
    const int nr = rs.count();
    const int64_t stride = w.nchunks + 1;
    // the super-chunks [lo, hi) of this call: all of them, or — one phase of a split
    // exchange, parts < ready landed — those every index of which has landed and that
    // no earlier phase took (landed_below is non-decreasing in the part)
    const int64_t nsc = ceil_div(w.nchunks, (int64_t)m), span = (int64_t)m * kChunk;
    int64_t lo = 0, hi = nsc;
    if (rs.parts > 1) {
        const int p = rs.ready - 1;
        if (p > 0) lo = rs.landed_below(p - 1) / span;
        if (p < rs.parts - 1) hi = rs.landed_below(p) / span;
        lo = lo < 0 ? 0 : (lo > nsc ? nsc : lo);
        hi = hi < lo ? lo : (hi > nsc ? nsc : hi);
    }
    const int64_t nwaves = (int64_t)gridDim.x * kSegWaves;
    for (int64_t sc0 = lo + (xcd_block(blockIdx.x, gridDim.x) * kSegWaves + wv) * kSCB; sc0 < hi;
         sc0 += nwaves * kSCB) {
        // run bounds at the kSCB + 1 super-chunk edges, lanes < nr (one run each)
        long long bb[kSCB + 1];
        uintptr_t rv = 0, ri = 0;
        if (lane < nr) {
            const Run run = rs.get(lane);
            rv = reinterpret_cast<uintptr_t>(run.vals);
            ri = reinterpret_cast<uintptr_t>(run.idx);
            const long long* bnd = w.bnd + (int64_t)lane * stride;
#pragma unroll
            for (int j = 0; j <= kSCB; ++j) {
                const int64_t c = (sc0 + j) * m < w.nchunks ? (sc0 + j) * m : w.nchunks;
                bb[j] = bnd[c];
            }
            long long prev = 0;
#pragma unroll
            for (int j = 0; j <= kSCB; ++j) {   // clamp: stale bounds of an unsorted run stay in range
                bb[j] = bb[j] < prev ? prev : (bb[j] > run.count ? run.count : bb[j]);
                prev = bb[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j <= kSCB; ++j) bb[j] = 0;
        }
        // Lane l takes entry l of each super-chunk: its run r = #{q : roff[q+1] <= l},
        // found with scalar run offsets (readlane) — no cross-lane shuffles.
        int T[kSCB], off[kSCB];
        float v[kSCB];
#pragma unroll
        for (int j = 0; j < kSCB; ++j) {
            const long long c64 = bb[j + 1] - bb[j];
            const int cnt = c64 > 65 ? 65 : (int)c64;   // > 64 entries overflow anyway
            int roff = 0, r = 0, first = 0;
            long long e0 = 0;
            uintptr_t pv = 0, pi = 0;
            for (int q = 0; q < nr; ++q) {   // uniform loop, scalar bookkeeping
                const int cq = __builtin_amdgcn_readlane(cnt, q);
                if (lane >= roff) {
                    r = q;
                    first = roff;
                }
                roff += cq;
            }
            T[j] = roff;
            for (int q = 0; q < nr; ++q) {
                const long long bq = ((long long)__builtin_amdgcn_readlane((int)(bb[j] >> 32), q) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)bb[j], q);
                const uintptr_t vq = ((uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)(rv >> 32), q) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)rv, q);
                const uintptr_t iq = ((uintptr_t)(uint32_t)__builtin_amdgcn_readlane((int)(ri >> 32), q) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)ri, q);
                if (r == q) {
                    e0 = bq;
                    pv = vq;
                    pi = iq;
                }
            }
            off[j] = -1;
            v[j] = 0.f;
            if (T[j] <= 64 && lane < T[j]) {
                const long long e = e0 + (lane - first);
                v[j] = load_val<VD>(reinterpret_cast<const void*>(pv), e);
                const long long i = load_idx<ID>(reinterpret_cast<const void*>(pi), e);
                const long long lo_i = (sc0 + j) * m * (long long)kChunk;
                const long long hi_i = (sc0 + j + 1) * m < w.nchunks ? (sc0 + j + 1) * m * (long long)kChunk : n;
                if (i >= lo_i && i < hi_i)
                    off[j] = (int)(i - lo_i);
                else
                    atomicOr(w.status, 2);   // only an unsorted run lands outside its chunks
            }
        }
#pragma unroll
        for (int j = 0; j < kSCB; ++j) {
            if (sc0 + j >= hi || T[j] == 0) continue;   // uniform
            if (T[j] > 64) {
                if (lane == 0) w.ovf_list[atomicAdd(w.ovf_cnt, 1)] = (int32_t)(sc0 + j);
                continue;
            }
            // an index in two runs (rare: ~W*ratio per entry) sets a bit another lane set
            bool dup = false;
            if (off[j] >= 0) {
                const uint32_t bit = 1u << (off[j] & 31);
                dup = (atomicOr(&bits[(off[j] & (kChunk - 1)) >> 5], bit) & bit) != 0;
            }
            const bool any_dup = __ballot(dup) != 0;
            if (off[j] >= 0) bits[(off[j] & (kChunk - 1)) >> 5] = 0;   // clean for the next super-chunk
            bool head = off[j] >= 0;
            float a = v[j];
            if (any_dup) {   // slow path: the first occurrence sums all of them in lane order
                a = 0.f;
                for (int q = 0; q < T[j]; ++q) {
                    const int oq = __shfl(off[j], q);
                    const float vq = __shfl(v[j], q);
                    if (head && oq == off[j]) {
                        if (q < lane)
                            head = false;
                        else
                            a = __fadd_rn(a, vq);
                    }
                }
            } else {
                a = __fadd_rn(0.f, a);   // index_put_ onto +0.0 (-0.0 -> +0.0)
            }
            // gran: an entry alone in its 64-B granule writes the whole granule (its value,
            // +0.0 around it — what the granule holds after the zero fill / re-zero):
            // full-granule stores instead of 4-B partial writes, 1.7x the line rate at 8M
            // lines (tools/scatterbench.hip). Shared granules (counted in LDS, mod kGranules,
            // so a false share only costs the fast path) keep the word store.
            // the granule must lie inside this super-chunk (which only this wave writes) and
            // inside grad: with an unaligned grad, granules straddle chunk edges
            const long long c_lo = (sc0 + j) * m * (long long)kChunk;
            const long long c_hi = (sc0 + j + 1) * m * (long long)kChunk < n ? (sc0 + j + 1) * m * (long long)kChunk : n;
            float* dst = grad + c_lo + off[j];
            const uintptr_t g = reinterpret_cast<uintptr_t>(dst) & ~(uintptr_t)63;
            const uint32_t gslot = (uint32_t)(g >> 6) & (kGranules - 1);
            if (gran && head) atomicAdd(&gcnt[gslot], 1u);
            if (gran) wave_sync_lds();
            const bool alone = gran && head && gcnt[gslot] == 1 && g >= reinterpret_cast<uintptr_t>(grad + c_lo) &&
                               g + 64 <= reinterpret_cast<uintptr_t>(grad + c_hi);
            const float val = scale != 1.0f ? __fmul_rn(a, scale) : a;
            if (alone) {
                const int pos = (int)((reinterpret_cast<uintptr_t>(dst) - g) >> 2);
                DGC_GLB f4v* g4 = (DGC_GLB f4v*)g;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f4v v = {0.f, 0.f, 0.f, 0.f};
                    if (pos >> 2 == q) v[pos & 3] = val;
                    g4[q] = v;
                }
            } else if (head) {
                *dst = val;
            }
            if (gran) {
                wave_sync_lds();
                if (head) gcnt[gslot] = 0;   // clean for the next super-chunk
            }
        }
    }
}

// The queued super-chunks, one 4096-element chunk per workgroup iteration.
template <int VD, int ID>
__global__ void __launch_bounds__(kBlock)
k_scatter_overflow(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale, int m) {
    const int64_t total = (int64_t)(*w.ovf_cnt) * m;
    for (int64_t q = blockIdx.x; q < total; q += gridDim.x) {
        const int64_t c = (int64_t)w.ovf_list[q / m] * m + q % m;
        if (c < w.nchunks) tile_chunk<VD, ID>(w, rs, grad, n, scale, c);
        __syncthreads();
    }
}

// ---------------------------------------------------------------- host side
static int vbytes(int vd) { return vd == DGC_F32 ? 4 : 2; }   // F16, BF16: 2
static int ibytes(int id) { return id == DGC_I32 ? 4 : 8; }

// words zeroed by the dense fill's first block (a null pointer with a zero count skips)
struct ZeroWords {
    int32_t* p[3];
    int32_t n[3];
};
int fill_zero(float* x, int64_t n, hipStream_t s, const ZeroWords& z);

// Sparse re-zero, the zero_() of a persistent output (dgc_decompress_packed_over):
// grad holds exactly the previous call's result over `prev`, so +0.0 everywhere but at
// prev's indices — zeroing those W*k slots is the whole-bucket fill for a fraction
// W*k/n of its traffic. Block (0, 0) also resets the scatter's status words.
template <int ID>
__global__ void __launch_bounds__(kBlock) k_clear_packed(RunSrc prev, float* __restrict__ grad, int64_t n,
                                                         ZeroWords z) {
    if (blockIdx.x == 0 && blockIdx.y == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
            for (int j = threadIdx.x; j < z.n[q]; j += kBlock) z.p[q][j] = 0;
    }
    // four lanes per entry zero the entry's whole 64-B granule (everything else in it
    // is +0.0 already, or another previous entry): full-granule stores, not 4-B partial
    // writes — 1.7x the line rate at 8M scattered lines (tools/scatterbench.hip)
    const Run run = prev.get_raw((int)blockIdx.y);
    const int part = (int)(threadIdx.x & 3);
    const uintptr_t lo = reinterpret_cast<uintptr_t>(grad), hi = reinterpret_cast<uintptr_t>(grad + n);
    for (long long t = (long long)blockIdx.x * kBlock + threadIdx.x; t < 4 * run.count;
         t += (long long)gridDim.x * kBlock) {
        const long long i = load_idx<ID>(run.idx, t >> 2);
        if (i < 0 || i >= n) continue;
        const uintptr_t g = reinterpret_cast<uintptr_t>(grad + i) & ~(uintptr_t)63;
        if (g >= lo && g + 64 <= hi)
            ((DGC_GLB f4v*)g)[part] = f4v{0.f, 0.f, 0.f, 0.f};
        else if (part == 0)
            grad[i] = 0.f;   // a granule that crosses the buffer's ends: the word alone
    }
}

// Decompress schedule. `entries` is a host-side upper bound on the total entries,
// `run_cap` on the entries of one run, and `runs` the number of runs when the host
// knows it (0 otherwise). dense: grad is first zeroed by dgc_fill_zero (one-shot
// 16-B stores, 7 TB/s — the fastest whole-line writer measured; tiles that also
// place the entries ran 0.69-1.2 ms against fill + scatter 0.61-0.98 ms at 1B,
// W = 1..8); then the sparse scatter:
//   one run          a thread per entry
//   several runs     bounds + a wave per kSCB super-chunks + the workgroup path for
//                    crowded super-chunks
// How grad is zeroed before the scatter (the reference's zero_()):
enum ZeroMode {
    kZeroNone,    // grad already +0.0 (dgc_fill_zero issued earlier): memset the status words
    kZeroDense,   // dense fill; its first block resets the status words
    kZeroPrev,    // re-zero the entries of `prev` (grad holds its result) + status words
    kZeroDone,    // dgc_clear_packed already did kZeroPrev's work on this workspace
};

static ZeroWords status_words(const DecWS& w) {
    return ZeroWords{{w.status, w.ovf_cnt, w.unsorted}, {1, 1, w.sort_cap ? kMaxRuns : 0}};
}

template <int ID>
static int launch_clear(const RunSrc& prev, const DecWS& w, float* grad, int64_t n, hipStream_t s) {
    const dim3 grid((unsigned)grid_for(4 * prev.capacity, kBlock, kMaxGrid / 2), (unsigned)prev.count());
    hipLaunchKernelGGL(k_clear_packed<ID>, grid, dim3(kBlock), 0, s, prev, grad, n, status_words(w));
    DGC_LAUNCHED();
    return DGC_OK;
}

// prev: the previous payload (kZeroPrev only). A phase of a split exchange (rs.parts >
// 1: the runs of part rs.ready - 1 just landed) bounds and regroups only those runs and
// scatters the super-chunks whose indices have all landed; zmode applies to phase 0.
template <int VD, int ID>
static int run_scatter(const DecWS& w, const RunSrc& rs, float* grad, int64_t n, float scale, int max_runs,
                       int zmode, int64_t entries, int64_t run_cap, int runs, hipStream_t s,
                       const RunSrc* prev = nullptr) {
    if (w.nchunks > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: n too large");
    const bool split = rs.payload && rs.parts > 1;
    const int part = split ? rs.ready - 1 : 0;
    // status, the overflow queue count and the unsorted flags are reset before any
    // kernel of this call can set them: by the dense fill's (or the sparse re-zero's)
    // first block, or memsets; a later phase of a split exchange only restarts the
    // overflow queue (the previous phase's queued super-chunks are done)
    if (part > 0) {
        DGC_HIP(hipMemsetAsync(w.ovf_cnt, 0, sizeof(int32_t), s));
    } else if (zmode == kZeroPrev) {
        DGC_TRY(launch_clear<ID>(*prev, w, grad, n, s));
    } else if (zmode == kZeroDense) {
        DGC_TRY(fill_zero(grad, n, s, status_words(w)));
    } else if (zmode == kZeroNone) {
        if (w.sort_cap) DGC_HIP(hipMemsetAsync(w.unsorted, 0, kMaxRuns * sizeof(int32_t), s));
        DGC_HIP(hipMemsetAsync(w.status, 0, sizeof(int32_t), s));
        DGC_HIP(hipMemsetAsync(w.ovf_cnt, 0, sizeof(int32_t), s));
    }
    if (runs == 1) {   // a thread per entry
        if (entries > 0) {
            hipLaunchKernelGGL((k_scatter_single<VD, ID>), dim3((unsigned)ceil_div(4 * entries, (int64_t)kBlock)),
                               dim3(kBlock), 0, s, w, rs, grad, n, scale);
            DGC_LAUNCHED();
        }
        return DGC_OK;
    }
    const unsigned bx = (unsigned)grid_for(run_cap + 1, kBlock, kMaxGrid / 2);
    const int ystep = split ? rs.parts : 1, yruns = split ? rs.world : max_runs;
    hipLaunchKernelGGL(k_bounds<ID>, dim3(bx, (unsigned)yruns), dim3(kBlock), 0, s, w, rs, n, run_cap, ystep, part);
    DGC_LAUNCHED();
    if (w.sort_cap) {
        if (run_cap > w.sort_cap) DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_decompress: run capacity above the regroup area");
        hipLaunchKernelGGL((k_regroup<VD, ID>), dim3((unsigned)yruns), dim3(kRegroupThreads), 0, s, w, rs, n, ystep,
                           part);
        DGC_LAUNCHED();
    }
    // super-chunk of m chunks holding ~32 entries on average
    int m = 1;
    const double per_chunk = (double)kChunk * (double)entries / (double)n;
    while (m < 64 && per_chunk * (2 * m) <= 32.0) m *= 2;
    const int64_t nsc = ceil_div(w.nchunks, (int64_t)m);
    // a split phase covers ~1/parts of the super-chunks (its waves loop over its window)
    const dim3 grid((unsigned)ceil_div(nsc, (int64_t)kSegWaves * kSCB * (split ? rs.parts : 1)));
    // whole-granule stores pay for their LDS bookkeeping from ~24 entries per chunk on
    // (measured at 1B: W = 8 scatter 0.39 -> 0.33 ms; W = 2 and 4 a few % slower with it)
    const int gran = per_chunk >= 24.0 ? 1 : 0;
    hipLaunchKernelGGL((k_scatter_waves<VD, ID>), grid, dim3(kBlock), 0, s, w, rs, grad, n, scale, m, gran);
    DGC_LAUNCHED();
    hipLaunchKernelGGL((k_scatter_overflow<VD, ID>), dim3(512), dim3(kBlock), 0, s, w, rs, grad, n, scale, m);
    DGC_LAUNCHED();
    return DGC_OK;
}

static int dispatch_scatter(int vd, int id, const DecWS& w, const RunSrc& rs, float* grad, int64_t n,
                            float scale, int max_runs, int dense, int64_t entries, int64_t run_cap, int runs,
                            hipStream_t s, const RunSrc* prev = nullptr) {
    if (vd == DGC_F32 && id == DGC_I64)
        return run_scatter<DGC_F32, DGC_I64>(w, rs, grad, n, scale, max_runs, dense, entries, run_cap, runs, s, prev);
    if (vd == DGC_F32 && id == DGC_I32)
        return run_scatter<DGC_F32, DGC_I32>(w, rs, grad, n, scale, max_runs, dense, entries, run_cap, runs, s, prev);
    if (vd == DGC_F16 && id == DGC_I64)
        return run_scatter<DGC_F16, DGC_I64>(w, rs, grad, n, scale, max_runs, dense, entries, run_cap, runs, s, prev);
    if (vd == DGC_F16 && id == DGC_I32)
        return run_scatter<DGC_F16, DGC_I32>(w, rs, grad, n, scale, max_runs, dense, entries, run_cap, runs, s, prev);
    DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress: unsupported value/index dtype (%d, %d)", vd, id);
}

static int check_common(int vd, int id, float* grad, int64_t n, void* ws, size_t ws_bytes, int runs,
                        int64_t sort_cap = 0) {
    if ((vd != DGC_F32 && vd != DGC_F16) || (id != DGC_I64 && id != DGC_I32))
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress: unsupported value/index dtype (%d, %d)", vd, id);
    if (!grad || n < 1) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: null grad or n < 1");
    if (runs < 1 || runs > kMaxRuns) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: 1..%d runs supported", kMaxRuns);
    size_t need = 0;
    carve_dec(nullptr, n, runs, sort_cap, &need);
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_decompress: workspace needs %zu bytes, 256-B aligned", need);
    return DGC_OK;
}

int decompress(const void* values, int vd, const void* indices, int id, int64_t total,
               const int64_t* run_offsets, int32_t nruns, float* grad, int64_t n, float scale, void* ws,
               size_t ws_bytes, hipStream_t s) {
    const int max_runs = run_offsets ? nruns : kMaxRuns;
    DGC_TRY(check_common(vd, id, grad, n, ws, ws_bytes, max_runs));
    if (total < 0 || (total > 0 && (!values || !indices)))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: null values/indices");
    DecWS w = carve_dec(ws, n, max_runs);
    DGC_HIP(hipMemsetAsync(w.nruns, 0, 4 * sizeof(int32_t), s));
    const char* v = static_cast<const char*>(values);
    const char* ix = static_cast<const char*>(indices);
    int known_runs = 0;
    if (run_offsets) {
        known_runs = nruns;
        HostRuns hr{};
        hr.n = nruns;
        for (int r = 0; r <= nruns; ++r) hr.off[r] = run_offsets[r];
        if (hr.off[0] != 0 || hr.off[nruns] != total)
            DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: run_offsets must span [0, total]");
        for (int r = 0; r < nruns; ++r)
            if (hr.off[r + 1] < hr.off[r]) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: run_offsets decrease");
        hipLaunchKernelGGL(k_runs_host, dim3(1), dim3(kMaxRuns), 0, s, w, hr, v, ix, vbytes(vd), ibytes(id));
        DGC_LAUNCHED();
    } else {
        if (total > 1) {
            if (id == DGC_I32)
                hipLaunchKernelGGL(k_find_descents<DGC_I32>, dim3(grid_for(total)), dim3(kBlock), 0, s, ix, total, w);
            else
                hipLaunchKernelGGL(k_find_descents<DGC_I64>, dim3(grid_for(total)), dim3(kBlock), 0, s, ix, total, w);
            DGC_LAUNCHED();
        }
        hipLaunchKernelGGL(k_runs_from_descents, dim3(1), dim3(64), 0, s, w, v, ix, vbytes(vd), ibytes(id), total);
        DGC_LAUNCHED();
        int32_t nr = 0;
        DGC_HIP(hipMemcpyAsync(&nr, w.nruns, sizeof(nr), hipMemcpyDeviceToHost, s));
        DGC_HIP(hipStreamSynchronize(s));
        if (nr == 0)
            DGC_FAIL(DGC_ERR_UNSORTED, "dgc_decompress: input has more than %d descending runs", kMaxRuns);
        known_runs = nr;
    }
    RunSrc rs{w.runs, w.nruns, nullptr, 0, 0, 0, 0, 0, nullptr, nullptr};
    return dispatch_scatter(vd, id, w, rs, grad, n, scale, max_runs, kZeroDense, total, total, known_runs, s);
}

int64_t payload_layout(int64_t capacity, int vd, int id, int64_t* voff, int64_t* ioff) {
    const int64_t v = 16;
    const int64_t i = (int64_t)align_up(v + capacity * vbytes(vd), 16);
    if (voff) *voff = v;
    if (ioff) *ioff = i;
    return (int64_t)align_up(i + capacity * ibytes(id), 256);
}

// ---------------------------------------------------------------- split exchange
// The allgather in `parts` collectives, so the scatter of what has landed runs while
// the rest is in flight (the W-dependent decompress under the exchange). A rank's
// packed payload is re-laid out as `parts` part buffers, each a packed payload of
// part_cap = ceil(capacity / parts) entries (dgc_payload_layout) whose header holds
// [0] its count and [1] the smallest index in the parts after it (INT64_MAX: none).
// Part p of every rank has landed => every entry below min_r bound(r, p) has: the
// scatter of phase p takes the super-chunks below that (and above phase p-1's).
constexpr int kMaxParts = 8;
constexpr int64_t kSplitScratch = 256;   // after the parts: per-part minima, arrival tickets

int64_t split_layout(int64_t capacity, int parts, int vd, int id, int64_t* part_cap, int64_t* voff, int64_t* ioff) {
    const int64_t pc = capacity > 0 ? ceil_div(capacity, (int64_t)parts) : 0;
    if (part_cap) *part_cap = pc;
    return payload_layout(pc, vd, id, voff, ioff);
}

// One pass over the payload's entries: each copied to its part, the per-part minimum
// index kept as max(~idx) (0 at rest: the scratch is zero between calls); the last
// workgroup writes the part headers and resets the scratch.
template <int VB, int IB>
__global__ void __launch_bounds__(kBlock)
k_payload_split(const char* __restrict__ src, int64_t cap, int64_t voff, int64_t ioff, char* __restrict__ dst,
                int parts, int64_t pc, int64_t pbytes, int64_t pvoff, int64_t pioff, uint64_t* pmin, uint32_t* tk) {
    __shared__ unsigned long long smin[kMaxParts];
    if (threadIdx.x < kMaxParts) smin[threadIdx.x] = 0;
    __syncthreads();
    long long cnt = *reinterpret_cast<const long long*>(src);
    cnt = cnt < 0 ? 0 : (cnt > cap ? cap : cnt);
    for (long long e = (long long)blockIdx.x * kBlock + threadIdx.x; e < cnt; e += (long long)gridDim.x * kBlock) {
        const int p = (int)(e / pc);
        const long long j = e - (long long)p * pc;
        char* part = dst + p * pbytes;
        long long idx;
        if (IB == 4) {
            const int32_t x = reinterpret_cast<const int32_t*>(src + ioff)[e];
            reinterpret_cast<int32_t*>(part + pioff)[j] = x;
            idx = x;
        } else {
            const int64_t x = reinterpret_cast<const int64_t*>(src + ioff)[e];
            reinterpret_cast<int64_t*>(part + pioff)[j] = x;
            idx = x;
        }
        if (VB == 2)
            reinterpret_cast<uint16_t*>(part + pvoff)[j] = reinterpret_cast<const uint16_t*>(src + voff)[e];
        else
            reinterpret_cast<uint32_t*>(part + pvoff)[j] = reinterpret_cast<const uint32_t*>(src + voff)[e];
        atomicMax(&smin[p], ~(unsigned long long)(idx < 0 ? 0 : idx));
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)parts && smin[threadIdx.x])
        __hip_atomic_fetch_max(reinterpret_cast<unsigned long long*>(pmin) + threadIdx.x, smin[threadIdx.x],
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!last_block_arrival8(tk, blockIdx.x, gridDim.x)) return;
    if (threadIdx.x == 0) {
        long long bound = LLONG_MAX;
        for (int p = parts - 1; p >= 0; --p) {
            long long* h = reinterpret_cast<long long*>(dst + p * pbytes);
            const long long c = cnt - (long long)p * pc;
            h[0] = c < 0 ? 0 : (c > pc ? pc : c);
            h[1] = bound;
            const uint64_t v = __hip_atomic_exchange(reinterpret_cast<unsigned long long*>(pmin) + p, 0ull,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const long long mn = v ? (long long)~v : LLONG_MAX;
            bound = mn < bound ? mn : bound;
        }
    }
}

int payload_split(const void* payload, int64_t capacity, int parts, int vd, int id, void* split, hipStream_t s) {
    if ((vd != DGC_F32 && vd != DGC_F16 && vd != DGC_BF16) || (id != DGC_I64 && id != DGC_I32))
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_payload_split: unsupported value/index dtype (%d, %d)", vd, id);
    if (!payload || !split || capacity < 0 || parts < 1 || parts > kMaxParts)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_payload_split: null buffer, capacity < 0 or parts outside 1..%d", kMaxParts);
    if ((reinterpret_cast<uintptr_t>(payload) | reinterpret_cast<uintptr_t>(split)) & 255)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_payload_split: buffers must be 256-B aligned");
    int64_t voff, ioff, pc, pvoff, pioff;
    payload_layout(capacity, vd, id, &voff, &ioff);
    const int64_t pbytes = split_layout(capacity, parts, vd, id, &pc, &pvoff, &pioff);
    char* dst = static_cast<char*>(split);
    auto* pmin = reinterpret_cast<uint64_t*>(dst + parts * pbytes);
    auto* tk = reinterpret_cast<uint32_t*>(pmin + kMaxParts);
    const unsigned g = (unsigned)grid_for(capacity, kBlock * 4);
    const char* src = static_cast<const char*>(payload);
    const int vb = vbytes(vd);
    if (pc == 0) {   // no entries: headers only
        DGC_HIP(hipMemsetAsync(dst, 0, (size_t)parts * pbytes, s));
        return DGC_OK;
    }
    if (vb == 2 && id == DGC_I32)
        hipLaunchKernelGGL((k_payload_split<2, 4>), dim3(g), dim3(kBlock), 0, s, src, capacity, voff, ioff, dst, parts, pc,
                           pbytes, pvoff, pioff, pmin, tk);
    else if (vb == 2)
        hipLaunchKernelGGL((k_payload_split<2, 8>), dim3(g), dim3(kBlock), 0, s, src, capacity, voff, ioff, dst, parts, pc,
                           pbytes, pvoff, pioff, pmin, tk);
    else if (id == DGC_I32)
        hipLaunchKernelGGL((k_payload_split<4, 4>), dim3(g), dim3(kBlock), 0, s, src, capacity, voff, ioff, dst, parts, pc,
                           pbytes, pvoff, pioff, pmin, tk);
    else
        hipLaunchKernelGGL((k_payload_split<4, 8>), dim3(g), dim3(kBlock), 0, s, src, capacity, voff, ioff, dst, parts, pc,
                           pbytes, pvoff, pioff, pmin, tk);
    DGC_LAUNCHED();
    return DGC_OK;
}

static RunSrc split_src(const void* gathered, int32_t world, int parts, int ready, int64_t pbytes, int64_t pc,
                        int64_t voff, int64_t ioff, const DecWS* w) {
    RunSrc r{nullptr, nullptr, static_cast<const char*>(gathered), pbytes, voff, ioff, pc, world,
             w ? w->unsorted : nullptr, w ? w->sorted : nullptr};
    r.parts = parts;
    r.ready = ready;
    r.pstride = (int64_t)world * pbytes;
    return r;
}

static int check_split(const void* gathered, int32_t world, int parts, int64_t capacity, int vd, int id,
                       const char* fn) {
    if (!gathered || world < 1 || parts < 2 || parts > kMaxParts || capacity < 0 || world * parts > kMaxRuns)
        DGC_FAIL(DGC_ERR_INVALID, "%s: null buffer, parts outside 2..%d or world * parts > %d", fn, kMaxParts, kMaxRuns);
    if ((vd != DGC_F32 && vd != DGC_F16) || (id != DGC_I64 && id != DGC_I32))
        DGC_FAIL(DGC_ERR_DTYPE, "%s: unsupported value/index dtype (%d, %d)", fn, vd, id);
    return DGC_OK;
}

// Phase `part` of the split decompress (parts < part landed and scattered by the
// earlier phases, in order, on this workspace). grad holds +0.0 (zeroed before phase 0
// — cleared: by dgc_clear_split on this workspace, which also reset its status words).
int scatter_split(const void* gathered, int32_t world, int parts, int part, int64_t capacity, int vd, int id,
                  float* grad, int64_t n, float scale, int cleared, void* ws, size_t ws_bytes, hipStream_t s) {
    DGC_TRY(check_split(gathered, world, parts, capacity, vd, id, "dgc_scatter_split"));
    if (part < 0 || part >= parts) DGC_FAIL(DGC_ERR_INVALID, "dgc_scatter_split: part %d outside 0..%d", part, parts - 1);
    int64_t pc, voff, ioff;
    const int64_t pbytes = split_layout(capacity, parts, vd, id, &pc, &voff, &ioff);
    DGC_TRY(check_common(vd, id, grad, n, ws, ws_bytes, world * parts, pc));
    const DecWS w = carve_dec(ws, n, world * parts, pc);
    const RunSrc rs = split_src(gathered, world, parts, part + 1, pbytes, pc, voff, ioff, &w);
    return dispatch_scatter(vd, id, w, rs, grad, n, scale, world * parts, cleared ? kZeroDone : kZeroNone,
                            (int64_t)world * parts * pc, pc, world * parts, s);
}

int clear_split(const void* prev, int32_t world, int parts, int64_t capacity, int vd, int id, float* grad, int64_t n,
                void* ws, size_t ws_bytes, hipStream_t s) {
    DGC_TRY(check_split(prev, world, parts, capacity, vd, id, "dgc_clear_split"));
    int64_t pc, voff, ioff;
    const int64_t pbytes = split_layout(capacity, parts, vd, id, &pc, &voff, &ioff);
    DGC_TRY(check_common(vd, id, grad, n, ws, ws_bytes, world * parts, pc));
    const DecWS w = carve_dec(ws, n, world * parts, pc);
    const RunSrc pr = split_src(prev, world, parts, parts, pbytes, pc, voff, ioff, nullptr);
    return id == DGC_I32 ? launch_clear<DGC_I32>(pr, w, grad, n, s) : launch_clear<DGC_I64>(pr, w, grad, n, s);
}

int decompress_packed(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity, int vd,
                      int id, float* grad, int64_t n, float scale, void* ws, size_t ws_bytes, hipStream_t s,
                      int zmode, const void* prev = nullptr) {
    DGC_TRY(check_common(vd, id, grad, n, ws, ws_bytes, world, capacity));
    int64_t voff, ioff;
    const int64_t min_stride = payload_layout(capacity, vd, id, &voff, &ioff);
    if (!payload || rank_stride < min_stride || capacity < 0)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_packed: rank_stride %lld < layout %lld",
                 (long long)rank_stride, (long long)min_stride);
    DecWS w = carve_dec(ws, n, world, capacity);
    RunSrc rs{nullptr, nullptr, static_cast<const char*>(payload), rank_stride, voff, ioff, capacity, world,
              w.unsorted, w.sorted};
    if (zmode == kZeroPrev) {
        if (prev == payload) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_packed_over: prev must be another buffer");
        const RunSrc pr{nullptr, nullptr, static_cast<const char*>(prev), rank_stride, voff, ioff, capacity, world,
                        nullptr, nullptr};
        return dispatch_scatter(vd, id, w, rs, grad, n, scale, world, zmode, (int64_t)world * capacity, capacity,
                                world, s, &pr);
    }
    return dispatch_scatter(vd, id, w, rs, grad, n, scale, world, zmode, (int64_t)world * capacity, capacity,
                            world, s);
}

// dgc_clear_packed: kZeroPrev's re-zero alone (see dgc_hip.h).
int clear_packed(const void* prev, int32_t world, int64_t rank_stride, int64_t capacity, int vd, int id,
                 float* grad, int64_t n, void* ws, size_t ws_bytes, hipStream_t s) {
    DGC_TRY(check_common(vd, id, grad, n, ws, ws_bytes, world, capacity));
    int64_t voff, ioff;
    const int64_t min_stride = payload_layout(capacity, vd, id, &voff, &ioff);
    if (!prev || rank_stride < min_stride || capacity < 0)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_clear_packed: null payload or rank_stride %lld < layout %lld",
                 (long long)rank_stride, (long long)min_stride);
    DecWS w = carve_dec(ws, n, world, capacity);
    const RunSrc pr{nullptr, nullptr, static_cast<const char*>(prev), rank_stride, voff, ioff, capacity, world,
                    nullptr, nullptr};
    return id == DGC_I32 ? launch_clear<DGC_I32>(pr, w, grad, n, s) : launch_clear<DGC_I64>(pr, w, grad, n, s);
}

// Zero fill (the sparse scatter's precondition): one-shot workgroups, one 16-B
// plain store per lane — measured 7.0 TB/s on MI355X at 4 GB, vs 5.2-6.2 for
// grid-stride or non-temporal forms (tools/membench.hip). Block 0 also zeroes the
// decompress's status words (ZeroWords), which saves the scatter two memset packets.
__global__ void __launch_bounds__(kBlock) k_fill_zero(float4* __restrict__ x, int64_t n4, ZeroWords z, int wt) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n4) st_stream(x + i, make_float4(0.f, 0.f, 0.f, 0.f), wt);
    if (blockIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q)
            for (int j = threadIdx.x; j < z.n[q]; j += kBlock) z.p[q][j] = 0;
    }
}

__global__ void k_fill_zero1(float* __restrict__ x, int64_t begin, int64_t n) {
    const int64_t i = begin + threadIdx.x;
    if (i < n) x[i] = 0.f;
}

// z: words to zero in the same launch (or their memsets when x gets no vector kernel).
int fill_zero(float* x, int64_t n, hipStream_t s, const ZeroWords& z) {
    if (!x || n < 0) DGC_FAIL(DGC_ERR_INVALID, "dgc_fill_zero: null buffer or n < 0");
    bool zeroed = false;
    if (n == 0) {
        for (int q = 0; q < 3; ++q)
            if (z.n[q]) DGC_HIP(hipMemsetAsync(z.p[q], 0, sizeof(int32_t) * z.n[q], s));
        return DGC_OK;
    }
    if (reinterpret_cast<uintptr_t>(x) & 3) DGC_FAIL(DGC_ERR_INVALID, "dgc_fill_zero: buffer must be 4-B aligned");
    // scalar head up to the first 16-B boundary (a grad that is an offset view), then 16-B stores
    const int64_t lead = std::min<int64_t>(n, (int64_t)((16 - (reinterpret_cast<uintptr_t>(x) & 15)) & 15) / 4);
    if (lead > 0) {
        hipLaunchKernelGGL(k_fill_zero1, dim3(1), dim3(64), 0, s, x, 0, lead);
        DGC_LAUNCHED();
        x += lead;
        n -= lead;
    }
    const int64_t n4 = n / 4;
    if (n4 > 0) {
        if (ceil_div(n4, (int64_t)kBlock) > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_fill_zero: n too large");
        hipLaunchKernelGGL(k_fill_zero, dim3((unsigned)ceil_div(n4, (int64_t)kBlock)), dim3(kBlock), 0, s,
                           reinterpret_cast<float4*>(x), n4, z, (int)write_through(4 * n4));
        DGC_LAUNCHED();
        zeroed = true;
    }
    if (!zeroed)
        for (int q = 0; q < 3; ++q)
            if (z.n[q]) DGC_HIP(hipMemsetAsync(z.p[q], 0, sizeof(int32_t) * z.n[q], s));
    const int64_t head = n4 * 4;
    if (head < n) {
        hipLaunchKernelGGL(k_fill_zero1, dim3(1), dim3(64), 0, s, x, head, n);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

}  // namespace dgc

// ---------------------------------------------------------------- sink bindings
// workspace -> host-mapped error words (dgc_decompress_bind_sink); looked up on the host
// when a call carves its workspace, so the kernels get the pointer as an argument.
namespace dgc {
namespace {
std::mutex g_sink_mu;
std::vector<std::pair<const void*, int32_t*>> g_sinks;
}  // namespace

int32_t* bound_sink(const void* ws) {
    std::lock_guard<std::mutex> lk(g_sink_mu);
    for (const auto& b : g_sinks)
        if (b.first == ws) return b.second;
    return nullptr;
}
}  // namespace dgc

extern "C" int dgc_decompress_bind_sink(const void* ws, int32_t* sink) {
    if (!ws) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_bind_sink: null workspace");
    std::lock_guard<std::mutex> lk(dgc::g_sink_mu);
    auto& v = dgc::g_sinks;
    for (size_t i = 0; i < v.size(); ++i)
        if (v[i].first == ws) {
            v.erase(v.begin() + (long)i);
            break;
        }
    if (sink) v.emplace_back(ws, sink);
    return DGC_OK;
}

extern "C" size_t dgc_decompress_packed_workspace(int64_t n, int32_t world, int64_t capacity) {
    size_t b = 0;
    dgc::carve_dec(nullptr, n, world, capacity, &b);
    return b;
}

extern "C" size_t dgc_decompress_workspace(int64_t n, int32_t max_runs) {
    size_t b = 0;
    if (max_runs < 1 || max_runs > dgc::kMaxRuns) max_runs = dgc::kMaxRuns;
    dgc::carve_dec(nullptr, n, max_runs, 0, &b);
    return b;
}

extern "C" int dgc_decompress(const void* values, int32_t vdtype, const void* indices, int32_t idtype,
                              int64_t total, const int64_t* run_offsets, int32_t nruns, float* grad,
                              int64_t n, float scale, void* ws, size_t ws_bytes, void* stream) {
    return dgc::decompress(values, vdtype, indices, idtype, total, run_offsets, nruns, grad, n, scale, ws,
                           ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_fill_zero(float* x, int64_t n, void* stream) {
    return dgc::fill_zero(x, n, static_cast<hipStream_t>(stream), dgc::ZeroWords{});
}

extern "C" int64_t dgc_payload_layout(int64_t capacity, int32_t vdtype, int32_t idtype,
                                      int64_t* values_offset, int64_t* indices_offset) {
    return dgc::payload_layout(capacity, vdtype, idtype, values_offset, indices_offset);
}

extern "C" int dgc_decompress_packed(const void* payload, int32_t world, int64_t rank_stride,
                                     int64_t capacity, int32_t vdtype, int32_t idtype, float* grad,
                                     int64_t n, float scale, void* ws, size_t ws_bytes, void* stream) {
    return dgc::decompress_packed(payload, world, rank_stride, capacity, vdtype, idtype, grad, n, scale, ws,
                                  ws_bytes, static_cast<hipStream_t>(stream), dgc::kZeroDense);
}

extern "C" int dgc_decompress_packed_over(const void* payload, const void* prev_payload, int32_t world,
                                          int64_t rank_stride, int64_t capacity, int32_t vdtype, int32_t idtype,
                                          float* grad, int64_t n, float scale, void* ws, size_t ws_bytes,
                                          void* stream) {
    if (!prev_payload) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_packed_over: null prev_payload");
    return dgc::decompress_packed(payload, world, rank_stride, capacity, vdtype, idtype, grad, n, scale, ws,
                                  ws_bytes, static_cast<hipStream_t>(stream), dgc::kZeroPrev, prev_payload);
}

extern "C" int dgc_clear_packed(const void* prev_payload, int32_t world, int64_t rank_stride, int64_t capacity,
                                int32_t vdtype, int32_t idtype, float* grad, int64_t n, void* ws, size_t ws_bytes,
                                void* stream) {
    return dgc::clear_packed(prev_payload, world, rank_stride, capacity, vdtype, idtype, grad, n, ws, ws_bytes,
                             static_cast<hipStream_t>(stream));
}

extern "C" int dgc_scatter_packed_cleared(const void* payload, int32_t world, int64_t rank_stride,
                                          int64_t capacity, int32_t vdtype, int32_t idtype, float* grad, int64_t n,
                                          float scale, void* ws, size_t ws_bytes, void* stream) {
    return dgc::decompress_packed(payload, world, rank_stride, capacity, vdtype, idtype, grad, n, scale, ws,
                                  ws_bytes, static_cast<hipStream_t>(stream), dgc::kZeroDone);
}

extern "C" int dgc_scatter_packed(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity,
                                  int32_t vdtype, int32_t idtype, float* grad, int64_t n, float scale, void* ws,
                                  size_t ws_bytes, void* stream) {
    return dgc::decompress_packed(payload, world, rank_stride, capacity, vdtype, idtype, grad, n, scale, ws,
                                  ws_bytes, static_cast<hipStream_t>(stream), dgc::kZeroNone);
}

extern "C" int64_t dgc_payload_split_layout(int64_t capacity, int32_t parts, int32_t vdtype, int32_t idtype,
                                            int64_t* part_capacity) {
    if (parts < 1 || parts > dgc::kMaxParts || capacity < 0) return 0;
    return dgc::split_layout(capacity, parts, vdtype, idtype, part_capacity, nullptr, nullptr);
}

extern "C" int64_t dgc_payload_split_bytes(int64_t capacity, int32_t parts, int32_t vdtype, int32_t idtype) {
    if (parts < 1 || parts > dgc::kMaxParts || capacity < 0) return 0;
    return parts * dgc::split_layout(capacity, parts, vdtype, idtype, nullptr, nullptr, nullptr) + dgc::kSplitScratch;
}

extern "C" int dgc_payload_split(const void* payload, int64_t capacity, int32_t parts, int32_t vdtype, int32_t idtype,
                                 void* split, void* stream) {
    return dgc::payload_split(payload, capacity, parts, vdtype, idtype, split, static_cast<hipStream_t>(stream));
}

extern "C" size_t dgc_decompress_split_workspace(int64_t n, int32_t world, int32_t parts, int64_t capacity) {
    if (parts < 1 || parts > dgc::kMaxParts || world < 1 || world * parts > dgc::kMaxRuns) return 0;
    size_t b = 0;
    dgc::carve_dec(nullptr, n, world * parts, capacity > 0 ? dgc::ceil_div(capacity, (int64_t)parts) : 0, &b);
    return b;
}

extern "C" int dgc_scatter_split(const void* gathered, int32_t world, int32_t parts, int32_t part, int64_t capacity,
                                 int32_t vdtype, int32_t idtype, float* grad, int64_t n, float scale, int32_t cleared,
                                 void* ws, size_t ws_bytes, void* stream) {
    return dgc::scatter_split(gathered, world, parts, part, capacity, vdtype, idtype, grad, n, scale, cleared, ws,
                              ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_clear_split(const void* prev_gathered, int32_t world, int32_t parts, int64_t capacity,
                               int32_t vdtype, int32_t idtype, float* grad, int64_t n, void* ws, size_t ws_bytes,
                               void* stream) {
    return dgc::clear_split(prev_gathered, world, parts, capacity, vdtype, idtype, grad, n, ws, ws_bytes,
                            static_cast<hipStream_t>(stream));
}

extern "C" int dgc_decompress_status(const void* ws, int32_t* status, void* stream) {
    if (!ws || !status) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_status: null argument");
    dgc::Carver c(const_cast<void*>(ws));
    c.take<dgc::Run>(dgc::kMaxRuns);
    int32_t* nr = c.take<int32_t>(4);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DGC_HIP(hipMemcpyAsync(status, nr + 1, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    DGC_HIP(hipStreamSynchronize(s));
    return DGC_OK;
}
