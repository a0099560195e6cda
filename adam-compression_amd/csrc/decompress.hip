// K6: deterministic decompress = grad.zero_().index_put_([idx], vals, accumulate=True)
// followed by grad.mul_(1/W) (dgc/compression.py:179-194), over the rank-order
// concatenation that the allgather produced (dgc/compression.py:200-212).
//
// The reference's single-threaded CPU index_put_ adds entries in input order. The
// input is a sequence of RUNS (one per rank; our compress emits each rank's indices
// ascending), so the dense result is reproduced bit-for-bit without atomics:
//
//   bounds  one thread per (run, chunk) binary-searches the first entry of the run
//           whose index reaches the chunk (runs are non-decreasing);
//   chunk   one workgroup per 4096-element chunk: zero a 16 KB LDS tile, add the
//           runs' entries for the chunk IN RUN ORDER (a barrier between runs; inside
//           a run an index appears once — or, for a non-decreasing run with
//           repeats, its first occurrence sums the repeats in order), scale by
//           1/W, and write the tile out with 16-B stores.
//
// HBM: the dense write (4 B/elem) plus the sparse reads W*k*(vb+ib). Untouched
// slots come out +0.0 exactly as zero_() * (1/W).
#include "dgc_common.hpp"

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
    int32_t* status;      // bit 0: index out of range
    int32_t* ndesc;       // detected descents
    int32_t* ovf_cnt;     // sparse scatter: super-chunks queued for the workgroup path
    int32_t* ovf_list;
    long long* desc;      // their positions (unsorted)
    long long* bnd;       // [kMaxRuns][nchunks + 1]
    int64_t nchunks;
};

static DecWS carve_dec(void* base, int64_t n, int32_t max_runs, size_t* bytes = nullptr) {
    Carver c(base);
    DecWS w{};
    w.nchunks = ceil_div(n, kChunk);
    w.runs = c.take<Run>(kMaxRuns);
    w.nruns = c.take<int32_t>(4);
    w.status = w.nruns ? w.nruns + 1 : nullptr;
    w.ndesc = w.nruns ? w.nruns + 2 : nullptr;
    w.ovf_cnt = w.nruns ? w.nruns + 3 : nullptr;
    w.desc = c.take<long long>(kMaxRuns);
    w.bnd = c.take<long long>((size_t)max_runs * (w.nchunks + 1));
    w.ovf_list = c.take<int32_t>(w.nchunks);
    if (bytes) *bytes = c.bytes();
    return w;
}

template <int VD>
__device__ __forceinline__ float load_val(const void* p, long long e) {
    if (VD == DGC_F16) return __half2float(reinterpret_cast<const __half*>(p)[e]);
    return reinterpret_cast<const float*>(p)[e];
}

template <int ID>
__device__ __forceinline__ long long load_idx(const void* p, long long e) {
    if (ID == DGC_I32) return reinterpret_cast<const int32_t*>(p)[e];
    return reinterpret_cast<const int64_t*>(p)[e];
}

// Where the runs come from: a table in the workspace (concatenated input), or the
// packed allgather buffer itself (rank r's header holds its count) — the latter
// needs no setup launch.
struct RunSrc {
    const Run* table;
    const int32_t* nruns_dev;
    const char* payload;          // packed mode when non-null
    int64_t stride, voff, ioff, capacity;
    int32_t world;
    __device__ __forceinline__ int count() const { return payload ? world : *nruns_dev; }
    __device__ __forceinline__ Run get(int r) const {
        if (!payload) return table[r];
        const char* base = payload + (int64_t)r * stride;
        long long c = *reinterpret_cast<const long long*>(base);
        c = c < 0 ? 0 : (c > capacity ? capacity : c);
        return Run{base + voff, base + ioff, c};
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
template <int ID>
__global__ void __launch_bounds__(kBlock)
k_bounds(DecWS w, RunSrc rs, int64_t n, int max_runs) {
    const int nr = rs.count();
    const int64_t stride = w.nchunks + 1;
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // set only by the next kernels
        *w.status = 0;
        *w.ovf_cnt = 0;
    }
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < (int64_t)max_runs * stride;
         t += (int64_t)gridDim.x * kBlock) {
        const int r = (int)(t / stride);
        if (r >= nr) break;
        const int64_t c = t - (int64_t)r * stride;
        const Run run = rs.get(r);
        const long long key = c == w.nchunks ? n : c * (long long)kChunk;
        long long lo = 0, hi = run.count;   // first entry with idx >= key
        while (lo < hi) {
            const long long mid = (lo + hi) >> 1;
            if (load_idx<ID>(run.idx, mid) < key)
                lo = mid + 1;
            else
                hi = mid;
        }
        w.bnd[t] = lo;
    }
}

// ---------------------------------------------------------------- chunk scatter
constexpr int kStage = 512;    // staged entries per chunk (avg 4*W at ratio 0.001); LDS ~21 KB -> 7 blocks/CU

__device__ __forceinline__ int lower_bound_lds(const int* a, int lo, int hi, int key) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// One workgroup per 4096-element chunk (one-shot grid). Phase 1 stages every run's
// entries for the chunk into LDS in one parallel load sweep (run order kept by
// position); phase 2 lets the FIRST occurrence of each index (in run order) add
// all of its occurrences in run order, from +0.0 — the sequential index_put_
// order — into the LDS tile; phase 3 scales and writes the tile with 16-B stores.
// Chunks with more than kStage entries fall back to one barrier per run.
// DENSE = false (sparse scatter): grad already holds +0.0 everywhere (zeroed by the
// caller, e.g. on a side stream while the compress and the allgather run), so only
// the indices present are written: the same sums, scaled, with no tile write.
template <int VD, int ID, bool DENSE>
__device__ void scatter_chunk(const DecWS& w, const RunSrc& rs, float* __restrict__ grad, int64_t n, float scale,
                              int64_t c) {
    __shared__ __attribute__((aligned(16))) float acc[kChunk];
    __shared__ int sidx[kStage];
    __shared__ float sval[kStage];
    __shared__ int roff[kMaxRuns + 1];
    __shared__ long long rb0[kMaxRuns];
    __shared__ const void* rval[kMaxRuns];
    __shared__ const void* ridx[kMaxRuns];
    const int nr = rs.count();
    const int64_t stride = w.nchunks + 1;
    const long long base = c * (long long)kChunk;
    const int tid = threadIdx.x, lane = tid & 63;
    if (c == 0 && tid < nr) {   // entries outside [0, n) are skipped: flag them
        const Run run = rs.get(tid);
        if (w.bnd[tid * stride] > 0 || w.bnd[tid * stride + w.nchunks] < run.count) atomicOr(w.status, 1);
    }
    float4* acc4 = reinterpret_cast<float4*>(acc);
    if (DENSE)
        for (int j = tid; j < kChunk / 4; j += kBlock) acc4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < 64) {   // run table for this chunk (nr <= 64: one wave)
        int cnt = 0;
        if (tid < nr) {
            const Run run = rs.get(tid);
            const long long b0 = w.bnd[tid * stride + c], b1 = w.bnd[tid * stride + c + 1];
            rb0[tid] = b0;
            rval[tid] = run.vals;
            ridx[tid] = run.idx;
            cnt = (int)(b1 - b0);
        }
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        if (tid < nr) roff[tid] = incl - cnt;
        if (tid == nr - 1) roff[nr] = incl;
    }
    __syncthreads();
    const int total = roff[nr];
    if (total <= kStage) {
        for (int t = tid; t < total; t += kBlock) {
            int r = 0;
            while (roff[r + 1] <= t) ++r;   // <= 64 runs, few entries: linear is fine
            const long long e = rb0[r] + (t - roff[r]);
            const long long i = load_idx<ID>(ridx[r], e) - base;
            sidx[t] = (i >= 0 && i < kChunk) ? (int)i : -1;
            sval[t] = load_val<VD>(rval[r], e);
        }
        __syncthreads();
        for (int t = tid; t < total; t += kBlock) {
            const int i = sidx[t];
            if (i < 0) {
                atomicOr(w.status, 2);   // only an unsorted run can land outside its chunk
                continue;
            }
            int r = 0;
            while (roff[r + 1] <= t) ++r;
            if (t > roff[r] && sidx[t - 1] == i) continue;   // repeat inside a non-decreasing run
            bool head = true;
            for (int q = 0; q < r && head; ++q) {
                const int p = lower_bound_lds(sidx, roff[q], roff[q + 1], i);
                head = !(p < roff[q + 1] && sidx[p] == i);
            }
            if (!head) continue;
            float a = 0.f;
            for (int q = r; q < nr; ++q) {
                for (int p = (q == r) ? t : lower_bound_lds(sidx, roff[q], roff[q + 1], i);
                     p < roff[q + 1] && sidx[p] == i; ++p)
                    a = __fadd_rn(a, sval[p]);
            }
            if (DENSE)
                acc[i] = a;
            else
                grad[base + i] = scale != 1.0f ? __fmul_rn(a, scale) : a;
        }
        if (!DENSE) return;
    } else {
        if (!DENSE) {   // rare (> kStage entries in one chunk): accumulate in LDS after all
            __syncthreads();
            for (int j = tid; j < kChunk / 4; j += kBlock) acc4[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            __syncthreads();
        }
        for (int r = 0; r < nr; ++r) {
            const long long b0 = rb0[r], b1 = rb0[r] + (roff[r + 1] - roff[r]);
            for (long long e = b0 + tid; e < b1; e += kBlock) {
                const long long i = load_idx<ID>(ridx[r], e);
                if (e > b0 && load_idx<ID>(ridx[r], e - 1) == i) continue;   // not the first of a repeat
                const long long off = i - base;
                if (off < 0 || off >= kChunk) {
                    atomicOr(w.status, 2);
                    continue;
                }
                float a = acc[off];
                long long f = e;
                do {
                    a = __fadd_rn(a, load_val<VD>(rval[r], f));
                    ++f;
                } while (f < b1 && load_idx<ID>(ridx[r], f) == i);
                acc[off] = a;
            }
            __syncthreads();
        }
        if (!DENSE) {   // write back the touched slots only (every entry rewrites its own)
            for (int r = 0; r < nr; ++r) {
                const long long b0 = rb0[r], b1 = rb0[r] + (roff[r + 1] - roff[r]);
                for (long long e = b0 + tid; e < b1; e += kBlock) {
                    const long long off = load_idx<ID>(ridx[r], e) - base;
                    if (off >= 0 && off < kChunk)
                        grad[base + off] = scale != 1.0f ? __fmul_rn(acc[off], scale) : acc[off];
                }
            }
            return;
        }
    }
    __syncthreads();
    const long long len = n - base < kChunk ? n - base : kChunk;
    if (aligned16(grad) && len == kChunk) {
        float4* g4 = reinterpret_cast<float4*>(grad + base);
        for (int j = tid; j < kChunk / 4; j += kBlock) {
            float4 v = acc4[j];
            if (scale != 1.0f) {
                v.x = __fmul_rn(v.x, scale);
                v.y = __fmul_rn(v.y, scale);
                v.z = __fmul_rn(v.z, scale);
                v.w = __fmul_rn(v.w, scale);
            }
            g4[j] = v;
        }
    } else {
        for (int j = tid; j < len; j += kBlock) grad[base + j] = scale != 1.0f ? __fmul_rn(acc[j], scale) : acc[j];
    }
}

template <int VD, int ID, bool DENSE>
__global__ void __launch_bounds__(kBlock)
k_scatter_chunks(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale) {
    scatter_chunk<VD, ID, DENSE>(w, rs, grad, n, scale, blockIdx.x);
}

// ---------------------------------------------------------------- sparse scatter
// grad holds +0.0 on entry (the reference's zero_(), done earlier); only the entries
// are written. The work scales with the entries, not with n.
//
// One run (W = 1): one thread per entry. The first of a repeat sums the repeats in
// order (index_put_ order); a descent or an index outside [0, n) sets the status.
template <int VD, int ID>
__global__ void __launch_bounds__(kBlock)
k_scatter_single(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale) {
    const Run run = rs.get(0);
    const long long j = (long long)blockIdx.x * kBlock + threadIdx.x;
    if (j >= run.count) return;
    const long long i = load_idx<ID>(run.idx, j);
    const long long ip = j > 0 ? load_idx<ID>(run.idx, j - 1) : -1;
    if (j > 0 && ip > i) atomicOr(w.status, 2);
    if (i < 0 || i >= n) {
        atomicOr(w.status, 1);
        return;
    }
    if (j > 0 && ip == i) return;   // not the first of a repeat
    float a = __fadd_rn(0.f, load_val<VD>(run.vals, j));
    for (long long f = j + 1; f < run.count && load_idx<ID>(run.idx, f) == i; ++f)
        a = __fadd_rn(a, load_val<VD>(run.vals, f));
    grad[i] = scale != 1.0f ? __fmul_rn(a, scale) : a;
}

// Several runs: one wave per super-chunk of m 4096-element chunks, m chosen on the
// host so a super-chunk holds ~32 entries. Lane l takes entry l of the super-chunk
// (runs concatenated in rank order, so lane order IS the index_put_ order); the
// lane holding the first occurrence of an index sums every occurrence in lane order
// through wave shuffles. A super-chunk with more than 64 entries is queued for the
// workgroup path (scatter_chunk per 4096-element chunk).
template <int VD, int ID>
__global__ void __launch_bounds__(kBlock)
k_scatter_waves(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale, int m) {
    const int lane = threadIdx.x & 63;
    const int64_t sc = (int64_t)blockIdx.x * kSegWaves + (threadIdx.x >> 6);
    const int64_t c0 = sc * m;
    if (c0 >= w.nchunks) return;
    const int64_t c1 = c0 + m < w.nchunks ? c0 + m : w.nchunks;
    const int nr = rs.count();
    const int64_t stride = w.nchunks + 1;
    long long b0 = 0, cnt = 0;
    if (lane < nr) {
        b0 = w.bnd[lane * stride + c0];
        cnt = w.bnd[lane * stride + c1] - b0;
        if (c0 == 0) {   // entries below 0 or at/after n are in no chunk: flag them once
            const Run run = rs.get(lane);
            if (b0 > 0 || w.bnd[lane * stride + w.nchunks] < run.count) atomicOr(w.status, 1);
        }
    }
    long long incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const long long T = __shfl(incl, nr - 1);
    if (T == 0) return;
    if (T > 64) {
        if (lane == 0) w.ovf_list[atomicAdd(w.ovf_cnt, 1)] = (int32_t)sc;
        return;
    }
    int r = 0;   // this lane's run: the number of runs ending at or before it
    for (int q = 0; q < nr; ++q) r += __shfl(incl, q) <= lane;
    r = r < nr ? r : nr - 1;
    const bool valid = lane < T;
    const long long first = __shfl(incl - cnt, r);   // shuffles with every lane active
    const long long e = __shfl(b0, r) + (lane - first);
    long long i = -1;
    float v = 0.f;
    if (valid) {
        const Run run = rs.get(r);
        i = load_idx<ID>(run.idx, e);
        v = load_val<VD>(run.vals, e);
    }
    bool head = valid;
    float a = 0.f;
    for (int q = 0; q < (int)T; ++q) {
        const long long iq = __shfl(i, q);
        const float vq = __shfl(v, q);
        if (valid && iq == i) {
            if (q < lane)
                head = false;
            else
                a = __fadd_rn(a, vq);
        }
    }
    if (!head) return;
    if (i < c0 * (long long)kChunk || i >= c1 * (long long)kChunk || i >= n) {
        atomicOr(w.status, 2);   // only an unsorted run lands outside its chunks
        return;
    }
    grad[i] = scale != 1.0f ? __fmul_rn(a, scale) : a;
}

// The queued super-chunks, one 4096-element chunk per workgroup iteration.
template <int VD, int ID>
__global__ void __launch_bounds__(kBlock)
k_scatter_overflow(DecWS w, RunSrc rs, float* __restrict__ grad, int64_t n, float scale, int m) {
    const int64_t total = (int64_t)(*w.ovf_cnt) * m;
    for (int64_t q = blockIdx.x; q < total; q += gridDim.x) {
        const int64_t c = (int64_t)w.ovf_list[q / m] * m + q % m;
        if (c < w.nchunks) scatter_chunk<VD, ID, false>(w, rs, grad, n, scale, c);
        __syncthreads();
    }
}

// ---------------------------------------------------------------- host side
static int vbytes(int vd) { return vd == DGC_F16 ? 2 : 4; }
static int ibytes(int id) { return id == DGC_I32 ? 4 : 8; }

int fill_zero(float* x, int64_t n, hipStream_t s);

// Decompress schedule. `entries` is a host-side upper bound on the total entries and
// `runs` the number of runs when the host knows it (0 otherwise).
//   dense, density > 1/16   one pass: LDS tiles, every element written once
//   dense, sparser          dgc_fill_zero (7 TB/s one-shot stores) + sparse scatter
//   sparse (grad pre-zeroed) sparse scatter only
// Sparse scatter: one run -> a thread per entry; several -> a wave per super-chunk.
template <int VD, int ID>
static int run_scatter(const DecWS& w, const RunSrc& rs, float* grad, int64_t n, float scale, int max_runs,
                       bool dense, int64_t entries, int runs, hipStream_t s) {
    if (w.nchunks > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: n too large");
    const double density = (double)entries / (double)n;
    if (dense && density > 1.0 / 16) {
        const int64_t work = (int64_t)max_runs * (w.nchunks + 1);
        hipLaunchKernelGGL(k_bounds<ID>, dim3(grid_for(work)), dim3(kBlock), 0, s, w, rs, n, max_runs);
        DGC_LAUNCHED();
        hipLaunchKernelGGL((k_scatter_chunks<VD, ID, true>), dim3((unsigned)w.nchunks), dim3(kBlock), 0, s, w,
                           rs, grad, n, scale);
        DGC_LAUNCHED();
        return DGC_OK;
    }
    if (dense) DGC_TRY(fill_zero(grad, n, s));
    if (runs == 1) {   // a thread per entry
        DGC_HIP(hipMemsetAsync(w.status, 0, sizeof(int32_t), s));
        if (entries > 0) {
            hipLaunchKernelGGL((k_scatter_single<VD, ID>), dim3((unsigned)ceil_div(entries, (int64_t)kBlock)),
                               dim3(kBlock), 0, s, w, rs, grad, n, scale);
            DGC_LAUNCHED();
        }
        return DGC_OK;
    }
    const int64_t work = (int64_t)max_runs * (w.nchunks + 1);
    hipLaunchKernelGGL(k_bounds<ID>, dim3(grid_for(work)), dim3(kBlock), 0, s, w, rs, n, max_runs);
    DGC_LAUNCHED();
    // super-chunk of m chunks holding ~32 entries on average
    int m = 1;
    const double per_chunk = (double)kChunk * density;
    while (m < 64 && per_chunk * (2 * m) <= 32.0) m *= 2;
    const int64_t nsc = ceil_div(w.nchunks, (int64_t)m);
    hipLaunchKernelGGL((k_scatter_waves<VD, ID>), dim3((unsigned)ceil_div(nsc, (int64_t)kSegWaves)), dim3(kBlock), 0,
                       s, w, rs, grad, n, scale, m);
    DGC_LAUNCHED();
    hipLaunchKernelGGL((k_scatter_overflow<VD, ID>), dim3(512), dim3(kBlock), 0, s, w, rs, grad, n, scale, m);
    DGC_LAUNCHED();
    return DGC_OK;
}

static int dispatch_scatter(int vd, int id, const DecWS& w, const RunSrc& rs, float* grad, int64_t n,
                            float scale, int max_runs, bool dense, int64_t entries, int runs, hipStream_t s) {
    if (vd == DGC_F32 && id == DGC_I64)
        return run_scatter<DGC_F32, DGC_I64>(w, rs, grad, n, scale, max_runs, dense, entries, runs, s);
    if (vd == DGC_F32 && id == DGC_I32)
        return run_scatter<DGC_F32, DGC_I32>(w, rs, grad, n, scale, max_runs, dense, entries, runs, s);
    if (vd == DGC_F16 && id == DGC_I64)
        return run_scatter<DGC_F16, DGC_I64>(w, rs, grad, n, scale, max_runs, dense, entries, runs, s);
    if (vd == DGC_F16 && id == DGC_I32)
        return run_scatter<DGC_F16, DGC_I32>(w, rs, grad, n, scale, max_runs, dense, entries, runs, s);
    DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress: unsupported value/index dtype (%d, %d)", vd, id);
}

static int check_common(int vd, int id, float* grad, int64_t n, void* ws, size_t ws_bytes, int runs) {
    if ((vd != DGC_F32 && vd != DGC_F16) || (id != DGC_I64 && id != DGC_I32))
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress: unsupported value/index dtype (%d, %d)", vd, id);
    if (!grad || n < 1) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: null grad or n < 1");
    if (runs < 1 || runs > kMaxRuns) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress: 1..%d runs supported", kMaxRuns);
    size_t need = 0;
    carve_dec(nullptr, n, runs, &need);
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
    RunSrc rs{w.runs, w.nruns, nullptr, 0, 0, 0, 0, 0};
    return dispatch_scatter(vd, id, w, rs, grad, n, scale, max_runs, true, total, known_runs, s);
}

int64_t payload_layout(int64_t capacity, int vd, int id, int64_t* voff, int64_t* ioff) {
    const int64_t v = 16;
    const int64_t i = (int64_t)align_up(v + capacity * vbytes(vd), 16);
    if (voff) *voff = v;
    if (ioff) *ioff = i;
    return (int64_t)align_up(i + capacity * ibytes(id), 256);
}

int decompress_packed(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity, int vd,
                      int id, float* grad, int64_t n, float scale, void* ws, size_t ws_bytes, hipStream_t s,
                      bool dense) {
    DGC_TRY(check_common(vd, id, grad, n, ws, ws_bytes, world));
    int64_t voff, ioff;
    const int64_t min_stride = payload_layout(capacity, vd, id, &voff, &ioff);
    if (!payload || rank_stride < min_stride || capacity < 0)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_packed: rank_stride %lld < layout %lld",
                 (long long)rank_stride, (long long)min_stride);
    DecWS w = carve_dec(ws, n, world);
    RunSrc rs{nullptr, nullptr, static_cast<const char*>(payload), rank_stride, voff, ioff, capacity, world};
    return dispatch_scatter(vd, id, w, rs, grad, n, scale, world, dense, (int64_t)world * capacity, world, s);
}

// Zero fill (the sparse scatter's precondition): one-shot workgroups, one 16-B
// plain store per lane — measured 7.0 TB/s on MI355X at 4 GB, vs 5.2-6.2 for
// grid-stride or non-temporal forms (tools/membench.hip).
__global__ void __launch_bounds__(kBlock) k_fill_zero(float4* __restrict__ x, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n4) x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ void k_fill_zero1(float* __restrict__ x, int64_t begin, int64_t n) {
    const int64_t i = begin + threadIdx.x;
    if (i < n) x[i] = 0.f;
}

int fill_zero(float* x, int64_t n, hipStream_t s) {
    if (!x || n < 0) DGC_FAIL(DGC_ERR_INVALID, "dgc_fill_zero: null buffer or n < 0");
    if (n == 0) return DGC_OK;
    if (!aligned16(x)) DGC_FAIL(DGC_ERR_INVALID, "dgc_fill_zero: buffer must be 16-B aligned");
    const int64_t n4 = n / 4;
    if (n4 > 0) {
        if (ceil_div(n4, (int64_t)kBlock) > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_fill_zero: n too large");
        hipLaunchKernelGGL(k_fill_zero, dim3((unsigned)ceil_div(n4, (int64_t)kBlock)), dim3(kBlock), 0, s,
                           reinterpret_cast<float4*>(x), n4);
        DGC_LAUNCHED();
    }
    const int64_t head = n4 * 4;
    if (head < n) {
        hipLaunchKernelGGL(k_fill_zero1, dim3(1), dim3(64), 0, s, x, head, n);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

}  // namespace dgc

extern "C" size_t dgc_decompress_workspace(int64_t n, int32_t max_runs) {
    size_t b = 0;
    if (max_runs < 1 || max_runs > dgc::kMaxRuns) max_runs = dgc::kMaxRuns;
    dgc::carve_dec(nullptr, n, max_runs, &b);
    return b;
}

extern "C" int dgc_decompress(const void* values, int32_t vdtype, const void* indices, int32_t idtype,
                              int64_t total, const int64_t* run_offsets, int32_t nruns, float* grad,
                              int64_t n, float scale, void* ws, size_t ws_bytes, void* stream) {
    return dgc::decompress(values, vdtype, indices, idtype, total, run_offsets, nruns, grad, n, scale, ws,
                           ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_fill_zero(float* x, int64_t n, void* stream) {
    return dgc::fill_zero(x, n, static_cast<hipStream_t>(stream));
}

extern "C" int64_t dgc_payload_layout(int64_t capacity, int32_t vdtype, int32_t idtype,
                                      int64_t* values_offset, int64_t* indices_offset) {
    return dgc::payload_layout(capacity, vdtype, idtype, values_offset, indices_offset);
}

extern "C" int dgc_decompress_packed(const void* payload, int32_t world, int64_t rank_stride,
                                     int64_t capacity, int32_t vdtype, int32_t idtype, float* grad,
                                     int64_t n, float scale, void* ws, size_t ws_bytes, void* stream) {
    return dgc::decompress_packed(payload, world, rank_stride, capacity, vdtype, idtype, grad, n, scale, ws,
                                  ws_bytes, static_cast<hipStream_t>(stream), true);
}

extern "C" int dgc_scatter_packed(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity,
                                  int32_t vdtype, int32_t idtype, float* grad, int64_t n, float scale, void* ws,
                                  size_t ws_bytes, void* stream) {
    return dgc::decompress_packed(payload, world, rank_stride, capacity, vdtype, idtype, grad, n, scale, ws,
                                  ws_bytes, static_cast<hipStream_t>(stream), false);
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
