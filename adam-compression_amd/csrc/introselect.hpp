// K5: exact emulation of torch's CPU topk(largest=True, sorted=False) for the
// resample branch: indices[topk(importance[indices], k)[1]] (dgc/compression.py:134-137).
//
// torch 2.10's CPU topk (aten/src/ATen/native/cpu/SortingKernel.cpp, topk_impl_loop)
// builds queue[j] = (x[j], j) and, for k * 64 > n, runs libstdc++'s
// std::nth_element(queue, queue + k - 1, queue + n, comp) with comp = "value greater"
// (NaN above everything); queue[0..k) IS the output, in that order — which boundary
// ties survive and the order of the transmitted (values, indices) both come from it.
// This file replays that introselect exactly, on one 512-thread workgroup:
//
//   while (last - first > 3):                     (depth limit 2*lg(n) -> heap select)
//     median of (first+1, mid, last-1) -> first   (std::__move_median_to_first)
//     cut = unguarded Hoare partition of [first+1, last) around *first
//     first = cut if cut <= nth else last = cut
//   insertion sort of the last <= 3
//
// The Hoare partition is done in parallel without replaying its scans: with P the
// pivot key, L_1 < L_2 < ... the positions in [first+1, last) with key <= P (where
// the left scan stops) and R_1 > R_2 > ... those in [first, last) with key >= P
// (where the right scan stops; the pivot slot stops it), the scans swap L_t <-> R_t
// exactly while L_t < R_t, and return cut = min(L_{s+1}, R_s) (R_0 = last): every
// swap leaves a stopper for each scan, so no scan passes the previous swap.
// L_t < R_t is "#(key >= P right of L_t) >= t" for a left stopper and "#(key <= P
// left of R_t) >= t" for a right stopper, so every element decides from two prefix
// counts whether it is swapped and with which rank; a pass writes the paired
// positions, the next pass swaps. oracle/introselect.py is the same algorithm in
// numpy, checked against torch.topk itself.
//
// Phases, by the size of the range still being partitioned:
//   > kNthGMinCand      (select.hip) in global memory by G co-resident workgroups per
//                       tensor, a barrier among them per pass (k_nth_global);
//   > kNthLds entries   in global memory (L2 / Infinity-Cache resident), 8 waves, each
//                       over a contiguous stretch, 8 tiles of loads in flight per lane;
//   > kNthWave entries  in LDS, same 8-wave step (four barriers per step);
//   <= kNthWave         one wave, wave-synchronous (no workgroup barrier at all).
// Entries are (key << 32 | j), key = |x| bits.
#pragma once

#include "dgc_common.hpp"

namespace dgc {

constexpr int kNthThreads = 512;    // 8 waves: 256 VGPRs per lane for the batched loads
constexpr int kNthWaves = kNthThreads / kWave;
constexpr int kNthLds = 12288;   // entries partitioned in LDS (96 KB + 48 KB of pair slots)
constexpr int kNthWave = 1024;   // entries finished by a single wave
constexpr int kNthPairLds = kNthLds / 2 + 1;            // LDS pair slots per side
constexpr int kNthMkLds = (kNthLds / 256 + 1) * 64;     // LDS-phase stopper bytes
// LDS of the one-workgroup replay, carved by the caller (k_nth_select shares it with K5b)
constexpr size_t kNthSmemBytes = (size_t)kNthLds * 8 + 2 * (size_t)kNthPairLds * 4 + kNthMkLds;

__device__ __forceinline__ uint32_t qkey(uint64_t e) { return (uint32_t)(e >> 32); }

#ifdef DGC_K5_PROF
// tools/k5_prof: phase timestamps (wall clock, 100 MHz) and step counts of the last
// K5 run by workgroup 0 — a profiling build only (make k5prof). Sub-phase sums and
// step counts accumulate in LDS (a global read-modify-write per sub-phase would put a
// memory round trip into every step it times) and reach g_k5prof once, at the end.
struct K5Prof {
    unsigned long long t[8];
    unsigned int steps[4];
    unsigned long long sub[8];   // global-phase step parts, summed over steps
    unsigned long long bt[64][8];   // per workgroup (tensor) < 64: the same stamps, [6] kernel end
    long long bn[64];               // its candidate count
    unsigned long long set[64][8];  // K5s k_resample_set per workgroup (tensor) < 64: phase ends
};
__device__ K5Prof g_k5prof;
__shared__ unsigned long long k5_lsub[8];
__shared__ unsigned int k5_lsteps[4];
#define K5_PROF_BEGIN() \
    do { if (threadIdx.x == 0) { for (int i_ = 0; i_ < 8; ++i_) k5_lsub[i_] = 0; \
         for (int i_ = 0; i_ < 4; ++i_) k5_lsteps[i_] = 0; } __syncthreads(); } while (0)
#define K5_PROF_END() \
    do { __syncthreads(); if (threadIdx.x == 0 && blockIdx.x == 0) { \
         for (int i_ = 0; i_ < 8; ++i_) g_k5prof.sub[i_] += k5_lsub[i_]; \
         for (int i_ = 0; i_ < 3; ++i_) g_k5prof.steps[i_] += k5_lsteps[i_]; } } while (0)
#define K5_STAMP(i) \
    do { if (threadIdx.x == 0) { const unsigned long long t_ = wall_clock64(); \
         if (blockIdx.x == 0) g_k5prof.t[i] = t_; \
         if (blockIdx.x < 64) g_k5prof.bt[blockIdx.x][i] = t_; } } while (0)
#define K5_STEP(i) \
    do { if (threadIdx.x == 0) k5_lsteps[i] += 1; } while (0)
// (in resample_set_body: the set's first workgroup, slot = tensor)
#define SET_STAMP(i) \
    do { if (threadIdx.x == 0 && b == 0 && t < 64) g_k5prof.set[t][i] = wall_clock64(); } while (0)
#define K5_SUB_BEGIN() unsigned long long k5_t0 = wall_clock64()
#define K5_SUB(i, global) \
    do { if ((global) && threadIdx.x == 0) { const unsigned long long t_ = wall_clock64(); \
         k5_lsub[i] += t_ - k5_t0; k5_t0 = t_; } } while (0)
// single-wave tail: sub[4] median, sub[5] loads + pairing, sub[6] swaps + cut
#define K5_WSUB_BEGIN() unsigned long long k5w_t0 = wall_clock64()
#define K5_WSUB_RESET() do { k5w_t0 = wall_clock64(); } while (0)
#define K5_WSUB(i) \
    do { if (threadIdx.x == 0) { const unsigned long long t_ = wall_clock64(); \
         k5_lsub[i] += t_ - k5w_t0; k5w_t0 = t_; } } while (0)
#else
#define K5_PROF_BEGIN() do { } while (0)
#define K5_PROF_END() do { } while (0)
#define K5_WSUB_BEGIN() do { } while (0)
#define K5_WSUB_RESET() do { } while (0)
#define K5_WSUB(i) do { } while (0)
#define K5_SUB_BEGIN() do { } while (0)
#define K5_SUB(i, global) do { } while (0)
#define K5_STAMP(i) do { } while (0)
#define K5_STEP(i) do { } while (0)
#define SET_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- heaps (depth limit)
// std::__adjust_heap + std::__push_heap on q[0..n) with comp = key greater (the
// heap's "largest" is the smallest key). Single thread.
template <class QP>
__device__ void nth_adjust_heap(QP q, int64_t hole, int64_t n, uint64_t v) {
    const int64_t top = hole;
    int64_t child = hole;
    while (child < (n - 1) / 2) {
        child = 2 * (child + 1);
        if (qkey(q[child]) > qkey(q[child - 1])) child--;
        q[hole] = q[child];
        hole = child;
    }
    if ((n & 1) == 0 && child == (n - 2) / 2) {
        child = 2 * (child + 1);
        q[hole] = q[child - 1];
        hole = child - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && qkey(q[parent]) > qkey(v)) {
        q[hole] = q[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    q[hole] = v;
}

// std::__heap_select(q, q + mid, q + n), then iter_swap(q, q + nth): the depth-limit
// exit of std::__introselect. Single thread; reached only by adversarial inputs.
template <class QP>
__device__ void nth_heap_select(QP q, int64_t mid, int64_t n, int64_t nth) {
    if (mid >= 2) {
        for (int64_t parent = (mid - 2) / 2;; --parent) {
            nth_adjust_heap(q, parent, mid, q[parent]);
            if (parent == 0) break;
        }
    }
    for (int64_t i = mid; i < n; ++i) {
        if (qkey(q[i]) > qkey(q[0])) {
            const uint64_t v = q[i];
            q[i] = q[0];
            nth_adjust_heap(q, 0, mid, v);
        }
    }
    const uint64_t t = q[0];
    q[0] = q[nth];
    q[nth] = t;
}

// std::__move_median_to_first(f, f+1, mid, l-1) with comp = key greater. One thread;
// the four entries are loaded together (one round trip when q is in global memory).
// Returns the pivot key.
template <class QP>
__device__ __forceinline__ uint32_t nth_median(QP q, int64_t f, int64_t l) {
    const int64_t a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const uint64_t ea = q[a], eb = q[b], ec = q[c], ef = q[f];
    const uint32_t ka = qkey(ea), kb = qkey(eb), kc = qkey(ec);
    int64_t m;
    uint64_t em;
    if (ka > kb) {
        if (kb > kc) { m = b; em = eb; }
        else if (ka > kc) { m = c; em = ec; }
        else { m = a; em = ea; }
    } else if (ka > kc) { m = a; em = ea; }
    else if (kb > kc) { m = c; em = ec; }
    else { m = b; em = eb; }
    q[m] = ef;   // m != f (a, b, c > f)
    q[f] = em;
    return qkey(em);
}

// std::__insertion_sort of q[f, l) (<= 3 entries after the loop). One thread.
template <class QP>
__device__ void nth_insertion_sort(QP q, int64_t f, int64_t l) {
    for (int64_t i = f + 1; i < l; ++i) {
        const uint64_t v = q[i];
        if (qkey(v) > qkey(q[f])) {
            for (int64_t j = i; j > f; --j) q[j] = q[j - 1];
            q[f] = v;
        } else {
            int64_t j = i - 1;
            while (qkey(v) > qkey(q[j])) {
                q[j + 1] = q[j];
                --j;
            }
            q[j + 1] = v;
        }
    }
}

// Lane's 4 consecutive entries of a 256-entry tile, positions in [begin, end). Tiles
// are laid from a 16-B-aligned base (nth_base), so a lane whose 4 entries are all in
// range reads them with two 16-B loads.
template <class QP>
__device__ __forceinline__ void nth_load4(QP q, int64_t e0, int64_t begin, int64_t end, uint64_t (&x)[4],
                                          uint32_t& valid) {
    if (e0 >= begin && e0 + 3 < end) {
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));   // no constructor: any address space
        const u64x2 a = *reinterpret_cast<rebind_t<QP, const u64x2>>(q + e0);
        const u64x2 b = *reinterpret_cast<rebind_t<QP, const u64x2>>(q + e0 + 2);
        x[0] = a[0];
        x[1] = a[1];
        x[2] = b[0];
        x[3] = b[1];
        valid = 0xFu;
        return;
    }
    valid = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool ok = e0 + j >= begin && e0 + j < end;
        x[j] = ok ? q[e0 + j] : 0ull;
        valid |= (uint32_t)ok << j;
    }
}

// The first tile position at or below a0 whose address is 16-B aligned.
template <class QP>
__device__ __forceinline__ int64_t nth_base(QP q, int64_t a0) {
    return a0 - (int64_t)((reinterpret_cast<uintptr_t>(q + a0) >> 3) & 1u);
}

// Pair slots: the positions (relative to f) of the t-th swapped left stopper L_t and of
// its partner R_t. Plain arrays (LDS phase, single-wave tail, multi-workgroup phase),
// or split (the one-workgroup global phase): slots t < cap in LDS, the rest in global
// memory — a 57k-candidate step swaps ~14k pairs, whose 4-B slot stores and loads
// were most of its time in global memory.
// fast / fl / fr: all slots below `end` in LDS (a uniform test), and the store there
// for element `on` of a lane — unconditional: an element that is no stopper writes the
// lane's word of a 64-word dummy instead. (A store under `if` became an exec-mask
// branch around it, four per tile in the pairing pass.)
template <class SP>
struct PlainSlotsT {
    SP l;
    SP r;
    SP d;   // the dummy words (LDS slots only)
    __device__ __forceinline__ void put_l(uint32_t t, uint32_t v) const { l[t] = v; }
    __device__ __forceinline__ void put_r(uint32_t t, uint32_t v) const { r[t] = v; }
    __device__ __forceinline__ uint32_t get_l(uint32_t t) const { return l[t]; }
    __device__ __forceinline__ uint32_t get_r(uint32_t t) const { return r[t]; }
    __device__ __forceinline__ bool fast(uint32_t) const { return true; }
    __device__ __forceinline__ bool gfast(uint32_t) const { return false; }
    __device__ __forceinline__ void gl_(bool, uint32_t, uint32_t) const {}
    __device__ __forceinline__ void gr_(bool, uint32_t, uint32_t) const {}
    __device__ __forceinline__ void fl(bool on, uint32_t t, uint32_t v) const {
        *(on ? l + t : d + (threadIdx.x & 63)) = v;
    }
    __device__ __forceinline__ void fr(bool on, uint32_t t, uint32_t v) const {
        *(on ? r + t : d + (threadIdx.x & 63)) = v;
    }
};

template <class SP>
__device__ __forceinline__ PlainSlotsT<SP> plain_slots(SP l, SP r, SP d = nullptr) { return PlainSlotsT<SP>{l, r, d}; }

struct SplitSlots {
    DGC_LDS uint32_t* ll;   // cap each
    DGC_LDS uint32_t* lr;
    uint32_t cap;
    DGC_GLB uint32_t* gl;   // indexed by t
    DGC_GLB uint32_t* gr;
    DGC_LDS uint32_t* d;    // the dummy words
    __device__ __forceinline__ void put_l(uint32_t t, uint32_t v) const {
        if (t < cap)
            ll[t] = v;
        else
            gl[t] = v;
    }
    __device__ __forceinline__ void put_r(uint32_t t, uint32_t v) const {
        if (t < cap)
            lr[t] = v;
        else
            gr[t] = v;
    }
    __device__ __forceinline__ uint32_t get_l(uint32_t t) const { return t < cap ? ll[t] : gl[t]; }
    __device__ __forceinline__ uint32_t get_r(uint32_t t) const { return t < cap ? lr[t] : gr[t]; }
    __device__ __forceinline__ bool fast(uint32_t end) const { return end <= cap; }
    // every slot from `begin` on is a global one: exec-masked global stores, no LDS / global
    // choice per element
    __device__ __forceinline__ bool gfast(uint32_t begin) const { return begin >= cap; }
    __device__ __forceinline__ void gl_(bool on, uint32_t t, uint32_t v) const {
        if (on) gl[t] = v;
    }
    __device__ __forceinline__ void gr_(bool on, uint32_t t, uint32_t v) const {
        if (on) gr[t] = v;
    }
    __device__ __forceinline__ void fl(bool on, uint32_t t, uint32_t v) const {
        *(on ? ll + t : d + (threadIdx.x & 63)) = v;
    }
    __device__ __forceinline__ void fr(bool on, uint32_t t, uint32_t v) const {
        *(on ? lr + t : d + (threadIdx.x & 63)) = v;
    }
};

// The step's swaps L_t <-> R_t, t < s (disjoint positions), by threads tid of nt:
// kNthSwapBatch pairs per thread with all their loads in flight before any store
// (8 for the global-memory phase, 2 in LDS where latency is short and registers count).
// left_only: the step's cut is above nth, so the introselect goes on in [f, cut) and
// never reads a position >= cut again (they are >= k: not output either) — every
// swapped R_t is >= cut, so only q[L_t] = q[R_t] is written (half the loads and stores).
template <int kNthSwapBatch, class Slots, class QP>
__device__ __forceinline__ void nth_swaps(QP q, const Slots& sl, int64_t f, uint32_t s, uint32_t tid,
                                          uint32_t nt, bool left_only = false) {
    for (uint32_t t0 = tid; t0 < s; t0 += nt * kNthSwapBatch) {
        uint32_t li[kNthSwapBatch], ri[kNthSwapBatch];
#pragma unroll
        for (int j = 0; j < kNthSwapBatch; ++j) {
            const uint32_t t = t0 + j * nt;
            li[j] = t < s ? sl.get_l(t) : 0u;
            ri[j] = t < s ? sl.get_r(t) : 0u;
        }
        uint64_t a[kNthSwapBatch], b[kNthSwapBatch];
#pragma unroll
        for (int j = 0; j < kNthSwapBatch; ++j) {
            if (t0 + j * nt < s) {
                if (!left_only) a[j] = q[f + li[j]];
                b[j] = q[f + ri[j]];
            }
        }
#pragma unroll
        for (int j = 0; j < kNthSwapBatch; ++j) {
            if (t0 + j * nt < s) {
                q[f + li[j]] = b[j];
                if (!left_only) q[f + ri[j]] = a[j];
            }
        }
    }
}

// The cut of a finished step (after its pass 2): min(first unswapped left stopper,
// last swapped right stopper), or the range end when nothing swapped.
__device__ __forceinline__ int64_t nth_cut(uint32_t s, unsigned long long r_min, unsigned long long l_next, int64_t l) {
    const int64_t rs = s ? (int64_t)r_min : l;
    const int64_t ln = l_next == ~0ull ? INT64_MAX : (int64_t)l_next;
    return ln < rs ? ln : rs;
}

__device__ __forceinline__ void stopper_masks(const uint64_t (&x)[4], uint32_t valid, uint32_t P, uint32_t& pl,
                                              uint32_t& pr) {
    pl = pr = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t k = qkey(x[j]);
        pl |= (uint32_t)(k <= P) << j;
        pr |= (uint32_t)(k >= P) << j;
    }
    pl &= valid;
    pr &= valid;
}

// Wave total of 4 predicate bits per lane (ballots: scalar, no cross-lane shuffles).
__device__ __forceinline__ uint32_t wave_count4(uint32_t p) {
    return (uint32_t)(__popcll(__ballot(p & 1u)) + __popcll(__ballot(p & 2u)) + __popcll(__ballot(p & 4u)) +
                      __popcll(__ballot(p & 8u)));
}

// The first element, in tile order 4 * lane + j, set in the per-j ballots m; 256 if none.
__device__ __forceinline__ uint32_t first_in_tile(const uint64_t (&m)[4]) {
    uint32_t best = 256;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (m[j]) {
            const uint32_t e = 4u * (uint32_t)__builtin_ctzll(m[j]) + (uint32_t)j;
            best = e < best ? e : best;
        }
    }
    return best;
}

// Pass 2 on one tile (elements tile + 4 * lane + j, stopper bits pl / pr from
// stopper_masks): ranks, pairing and the paired positions. runl / runr: the left and right stoppers before the tile; lpos/rpos
// hold positions relative to f. The step's results: paired (swaps), lnext (first
// unswapped left stopper), rmin (smallest swapped right stopper); INT64_MAX = none.
// BALLOT: accumulated wave-uniformly from ballots (a few tiles: no reduction after);
// else per lane, for the caller to reduce once after many tiles.
template <bool BALLOT, class Slots>
__device__ __forceinline__ void pair_tile(uint32_t pl, uint32_t pr, int64_t tile, int64_t f, uint32_t TR,
                                          uint32_t& runl, uint32_t& runr, const Slots& sl,
                                          uint32_t& paired, uint32_t& lnext, uint32_t& rmin) {
    // positions relative to f (32-bit: a range is < 2^32 entries); lnext / rmin too,
    // UINT32_MAX = none
    const int lane = threadIdx.x & 63;
    const uint32_t rel0 = (uint32_t)(tile - f) + 4u * (uint32_t)lane;
    uint32_t bl, tl, br, tr;
    wave_prefix4(pl, bl, tl);
    wave_prefix4(pr, br, tr);
    uint32_t rl = runl + bl;   // left stoppers before this element
    uint32_t rr = runr + br;   // right stoppers in [f+1, this element)
    if (!BALLOT) {
        // Whole-tile cases (wave-uniform): with every right stopper after the tile
        // outnumbering the left stoppers up to its end, all its left stoppers are
        // swapped and none of its right ones; with the left stoppers before it
        // outnumbering every right stopper from its start, the reverse. Only the tile(s)
        // where the two counts cross need the per-element test below. (Measured: a
        // third off the pairing pass; no gain in the few-tile single-wave tail.)
        const int64_t after = (int64_t)TR - runr - tr, from = (int64_t)TR - runr;
        if (after >= (int64_t)runl + tl) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if ((pl >> j) & 1u) sl.put_l(rl++, rel0 + (uint32_t)j);
            }
            paired += (uint32_t)__popc(pl);
            runl += tl;
            runr += tr;
            return;
        }
        if ((int64_t)runl >= from) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t i = rel0 + (uint32_t)j;
                if ((pr >> j) & 1u) {
                    rr += 1;
                    sl.put_r(TR - rr, i);
                    rmin = i < rmin ? i : rmin;
                }
                if (((pl >> j) & 1u) && i < lnext) lnext = i;
            }
            runl += tl;
            runr += tr;
            return;
        }
    }
    uint64_t msl[4], mln[4], msr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool isl = (pl >> j) & 1u, isr = (pr >> j) & 1u;
        const uint32_t i = rel0 + (uint32_t)j;
        const uint32_t rr_incl = rr + (isr ? 1u : 0u);
        // L_{rl+1} = i is swapped iff #(key >= P in (i, l)) >= rl + 1
        const bool swl = isl && TR - rr_incl >= rl + 1;
        // R_{u+1} = i with u = #(key >= P in (i, l)); swapped iff #(key <= P in [f+1, i)) >= u + 1
        const uint32_t u = TR - rr_incl;
        const bool swr = isr && rl >= u + 1;
        if (swl) sl.put_l(rl, i);
        if (swr) sl.put_r(u, i);
        if (BALLOT) {
            msl[j] = __ballot(swl);
            mln[j] = __ballot(isl && !swl);
            msr[j] = __ballot(swr);
        } else {
            paired += swl;
            if (isl && !swl && i < lnext) lnext = i;
            if (swr && i < rmin) rmin = i;
        }
        rl += isl;
        rr = rr_incl;
    }
    if (BALLOT) {
        paired += (uint32_t)(__popcll(msl[0]) + __popcll(msl[1]) + __popcll(msl[2]) + __popcll(msl[3]));
        const uint32_t el = first_in_tile(mln), er = first_in_tile(msr);
        const uint32_t t32 = (uint32_t)(tile - f);
        if (el < 256 && t32 + el < lnext) lnext = t32 + el;
        if (er < 256 && t32 + er < rmin) rmin = t32 + er;
    }
    runl += tl;
    runr += tr;
}


// ---------------------------------------------------------------- workgroup step
struct NthShared {
    int64_t f, l, depth;
    uint32_t pivot;                          // the step's pivot key (set by nth_median)
    uint32_t wl[kNthWaves], wr[kNthWaves];   // per-wave stopper counts
    uint32_t s;                              // swaps
    unsigned long long l_next, r_min;
    int heap_exit;
};

// One partition step over q[f, l) by the whole workgroup; the pivot is already at
// q[f] and sh.s / l_next / r_min are reset. On return (after the last barrier) the
// step's swaps are done and sh.s / l_next / r_min hold its result. Pass 1 keeps each
// lane's stopper bits of each tile in mk (one byte, LDS) when the step's tiles fit
// mk_tiles, so pass 2 reads bytes instead of the entries; otherwise it reloads them.
template <int kNthBatch, int kSwapBatch, class Slots, class QP, class MP>
__device__ void nth_step_wg(QP q, const Slots& sl, NthShared& sh, MP mk, int64_t mk_tiles, int64_t nth) {
    const int64_t f = uniform64(sh.f), l = uniform64(sh.l);
    const int lane = threadIdx.x & 63, wv = wave_id();
    const uint32_t P = uniform32(sh.pivot);
    const int64_t a0 = f + 1, base = nth_base(q, a0), R = l - base;
    const int64_t per = ceil_div(ceil_div(R, (int64_t)kNthWaves), (int64_t)256) * 256;
    const int64_t wb = base + wv * per, we = wb + per < l ? wb + per : l;
    const bool keep = ceil_div(R, (int64_t)256) <= mk_tiles;
    K5_SUB_BEGIN();
    // pass 1: stopper counts per wave, kNthBatch tiles of loads in flight per lane
    uint32_t cl = 0, cr = 0;
    for (int64_t t0 = wb; t0 < we; t0 += 256 * kNthBatch) {
        uint64_t x[kNthBatch][4];
        uint32_t valid[kNthBatch];
#pragma unroll
        for (int b = 0; b < kNthBatch; ++b) nth_load4(q, t0 + b * 256 + 4 * lane, a0, we, x[b], valid[b]);
#pragma unroll
        for (int b = 0; b < kNthBatch; ++b) {
            uint32_t pl, pr;
            stopper_masks(x[b], valid[b], P, pl, pr);
            cl += __popc(pl);
            cr += __popc(pr);
            if (keep && t0 + b * 256 < we) mk[((t0 + b * 256 - base) >> 8) * 64 + lane] = (uint8_t)(pl | (pr << 4));
        }
    }
    cl = wave_sum(cl);
    cr = wave_sum(cr);
    if (lane == 0) {
        sh.wl[wv] = cl;
        sh.wr[wv] = cr;
    }
    __syncthreads();
    K5_SUB(0, kNthBatch == 8);
    // every wave derives its own prefix and the total from the 16 wave counts
    uint32_t runl = 0, runr = 0, TR = 0;
#pragma unroll
    for (int i = 0; i < kNthWaves; ++i) {
        const uint32_t a = sh.wl[i], b = sh.wr[i];
        runl += i < wv ? a : 0u;
        runr += i < wv ? b : 0u;
        TR += b;
    }
    runl = uniform32(runl);
    runr = uniform32(runr);
    TR = uniform32(TR);
    // pass 2: ranks, pairing, paired positions
    uint32_t paired = 0, lnext = UINT32_MAX, rmin = UINT32_MAX;
    if (keep) {
        // Whole-tile cases from the tile's ballots (wave-uniform; pair_tile's reasoning):
        // a left-swap tile (all its left stoppers swapped, none of its right) ranks only
        // its left stoppers, a right-swap tile only its right ones, a tile between them
        // (neither side swapped) only feeds l_next; only the crossing tile(s) take the
        // per-element test. lnext_u / rmin_u: the wave's first such position (tiles go up).
        uint32_t paired_u = 0, lnext_u = UINT32_MAX, rmin_u = UINT32_MAX;
        const uint32_t below[4] = {0u, 1u, 3u, 7u};
#ifdef DGC_K5_PROF
        const unsigned long long k5_loop0 = wall_clock64();
        uint32_t k5_mixed = 0;
#endif
        for (int64_t t0 = wb; t0 < we; t0 += 256) {
            const uint32_t m = mk[((t0 - base) >> 8) * 64 + lane];
            const uint32_t pl = m & 15u, pr = m >> 4;
            uint64_t bl[4], br[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bl[j] = __ballot((pl >> j) & 1u);
                br[j] = __ballot((pr >> j) & 1u);
            }
            const uint32_t tl = (uint32_t)(__popcll(bl[0]) + __popcll(bl[1]) + __popcll(bl[2]) + __popcll(bl[3]));
            const uint32_t tr = (uint32_t)(__popcll(br[0]) + __popcll(br[1]) + __popcll(br[2]) + __popcll(br[3]));
            const uint32_t t32 = (uint32_t)(t0 - f), rel0 = t32 + 4u * (uint32_t)lane;
            const int64_t after = (int64_t)TR - runr - tr, from = (int64_t)TR - runr;
            if (after >= (int64_t)runl + tl) {
                if (tl) {
                    const uint32_t r0 = runl + ((mbcnt64(bl[0], 0u) + mbcnt64(bl[1], 0u)) +
                                                (mbcnt64(bl[2], 0u) + mbcnt64(bl[3], 0u)));
                    if (sl.fast(runl + tl)) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) sl.fl((pl >> j) & 1u, r0 + __popc(pl & below[j]), rel0 + (uint32_t)j);
                    } else if (sl.gfast(runl)) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) sl.gl_((pl >> j) & 1u, r0 + __popc(pl & below[j]), rel0 + (uint32_t)j);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if ((pl >> j) & 1u) sl.put_l(r0 + __popc(pl & below[j]), rel0 + (uint32_t)j);
                    }
                    paired_u += tl;
                }
            } else if ((int64_t)runl >= from) {
                if (tr) {
                    // R at rank rr (1-based, from f) takes slot TR - rr
                    const uint32_t r0 = runr + ((mbcnt64(br[0], 0u) + mbcnt64(br[1], 0u)) +
                                                (mbcnt64(br[2], 0u) + mbcnt64(br[3], 0u)));
                    if (sl.fast((uint32_t)from)) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            sl.fr((pr >> j) & 1u, TR - 1u - r0 - __popc(pr & below[j]), rel0 + (uint32_t)j);
                    } else if (sl.gfast((uint32_t)(from - tr))) {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            sl.gr_((pr >> j) & 1u, TR - 1u - r0 - __popc(pr & below[j]), rel0 + (uint32_t)j);
                    } else {
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if ((pr >> j) & 1u) sl.put_r(TR - 1u - r0 - __popc(pr & below[j]), rel0 + (uint32_t)j);
                    }
                    if (rmin_u == UINT32_MAX) rmin_u = t32 + first_in_tile(br);
                }
                if (tl && lnext_u == UINT32_MAX) lnext_u = t32 + first_in_tile(bl);
            } else if (after + tr < (int64_t)runl + 1 && (int64_t)runl + tl < after + 1) {
                if (tl && lnext_u == UINT32_MAX) lnext_u = t32 + first_in_tile(bl);
            } else {
                pair_tile<false>(pl, pr, t0, f, TR, runl, runr, sl, paired, lnext, rmin);
#ifdef DGC_K5_PROF
                k5_mixed += 1;
#endif
                continue;
            }
            runl += tl;
            runr += tr;
        }
#ifdef DGC_K5_PROF
        if (kNthBatch == 8 && blockIdx.x == 0 && lane == 0) {   // sub[7]: wave 0's tile loop; steps[3]: mixed tiles
            if (wv == 0) g_k5prof.sub[7] += wall_clock64() - k5_loop0;
            atomicAdd(&g_k5prof.steps[3], k5_mixed);
        }
#endif
        // fold the uniform results into lane 0's (reduced below)
        if (lane == 0) {
            paired += paired_u;
            lnext = lnext_u < lnext ? lnext_u : lnext;
            rmin = rmin_u < rmin ? rmin_u : rmin;
        }
    } else {
        for (int64_t t0 = wb; t0 < we; t0 += 256 * kNthBatch) {
            uint64_t x[kNthBatch][4];
            uint32_t valid[kNthBatch];
#pragma unroll
            for (int b = 0; b < kNthBatch; ++b) nth_load4(q, t0 + b * 256 + 4 * lane, a0, we, x[b], valid[b]);
#pragma unroll
            for (int b = 0; b < kNthBatch; ++b) {
                uint32_t pl, pr;
                stopper_masks(x[b], valid[b], P, pl, pr);
                pair_tile<false>(pl, pr, t0 + b * 256, f, TR, runl, runr, sl, paired, lnext, rmin);
            }
        }
    }
    paired = wave_sum(paired);
    lnext = wave_min_u32(lnext);
    rmin = wave_min_u32(rmin);
    if (lane == 0) {
        if (paired) atomicAdd(&sh.s, paired);
        if (lnext != UINT32_MAX) atomicMin(&sh.l_next, (unsigned long long)(f + lnext));
        if (rmin != UINT32_MAX) atomicMin(&sh.r_min, (unsigned long long)(f + rmin));
    }
    __syncthreads();
    K5_SUB(1, kNthBatch == 8);
    // pass 3: the swaps L_t <-> R_t, t < s (disjoint positions); only the left half of
    // each when the introselect goes on left of the cut
    const bool left_only = nth_cut(sh.s, sh.r_min, sh.l_next, l) > nth;
    nth_swaps<kSwapBatch>(q, sl, f, sh.s, threadIdx.x, kNthThreads, left_only);
    __syncthreads();
    K5_SUB(2, kNthBatch == 8);
}

// Thread 0, after a step: the cut and the next range.
__device__ __forceinline__ void nth_advance(NthShared& sh, int64_t nth) {
    const int64_t cut = nth_cut(sh.s, sh.r_min, sh.l_next, sh.l);
    if (cut <= nth)
        sh.f = cut;
    else
        sh.l = cut;
}

// The introselect loop on q[f, l) by the whole workgroup while the range exceeds
// `stop` entries; ends with a barrier, sh.f/l/depth updated or sh.heap_exit set.
// GLOBAL (the one-workgroup global-memory phase): mk_arena (arena_bytes of LDS) holds
// the step's stopper bytes and, after them, as many LDS pair slots as fit (the rest
// in gpos_l / gpos_r); otherwise mk / mk_tiles and the plain LDS slots lpos / rpos.
// Pointers typed by address space (dgc_common.hpp: DGC_GLB / DGC_LDS).
template <int kNthBatch, int kSwapBatch, bool GLOBAL, class QP, class SP>
__device__ __forceinline__ void nth_loop_wg(QP q, SP lpos, SP rpos, NthShared& sh, int64_t nth, int64_t stop,
                            DGC_LDS uint8_t* mk, int64_t mk_tiles, size_t arena_bytes = 0) {
    // thread 0 prepares a step: depth check, median, reset of the step's results
    auto prepare = [&]() -> bool {
        if (sh.l - sh.f <= stop) return false;
        if (sh.depth == 0) {
            nth_heap_select(q + sh.f, nth + 1 - sh.f, sh.l - sh.f, nth - sh.f);
            sh.heap_exit = 1;
            return false;
        }
        sh.depth -= 1;
        sh.pivot = nth_median(q, sh.f, sh.l);
        sh.s = 0;
        sh.l_next = ~0ull;
        sh.r_min = ~0ull;
        return true;
    };
    __shared__ int go;
    __shared__ uint32_t dummy[kWave];   // the unconditional slot stores' sink (PlainSlotsT::fl)
    if (threadIdx.x == 0) go = !sh.heap_exit && prepare();
    __syncthreads();
    while (go) {
        K5_STEP(stop == kNthLds ? 0 : 1);
        if constexpr (GLOBAL) {
            // the step's stopper bytes first (one per lane per 256-entry tile), then slots
            const int64_t tiles = (sh.l - sh.f) / 256 + 2;
            const size_t mk_bytes = (size_t)tiles * 64 <= arena_bytes / 2 ? (size_t)tiles * 64 : 0;
            const size_t off = (mk_bytes + 15) & ~(size_t)15;
            const uint32_t cap = (uint32_t)((arena_bytes - off) / 8);
            DGC_LDS uint32_t* ll = reinterpret_cast<DGC_LDS uint32_t*>(mk + off);
            const SplitSlots sl{ll, ll + cap, cap, lpos, rpos, lds(dummy)};
            nth_step_wg<kNthBatch, kSwapBatch>(q, sl, sh, mk, mk_bytes ? tiles : 0, nth);
        } else {
            nth_step_wg<kNthBatch, kSwapBatch>(q, plain_slots(lpos, rpos, lds(dummy)), sh, mk, mk_tiles, nth);
        }
        K5_SUB_BEGIN();
        if (threadIdx.x == 0) {
            nth_advance(sh, nth);
            go = prepare();
        }
        __syncthreads();
        K5_SUB(3, kNthBatch == 8);
    }
}

// ---------------------------------------------------------------- single-wave tail
// The same step by one wave on an LDS range of <= kNthWave entries, wave-synchronous
// (no workgroup barrier), with as few dependent LDS round trips as the step allows —
// a single wave's latency chain is the tail's whole cost:
//   1. every tile of the range loaded at once (<= 5 x 4 entries per lane, registers);
//   2. from the tiles' ballots alone, every element's swap test (pair_tile's: L_{rl+1}
//      swapped iff #(key >= P right of it) >= rl + 1; R with u stoppers right of it
//      iff rl >= u + 1), so s, L_{s+1} and R_s come from ballots, not from a search;
//   3. each swapped element stores its ENTRY (from registers) at its pair slot (xl[t]
//      for L_t, xr[u] for R_u: one store, the two tests exclude each other);
//   4. each swapped element loads its partner's entry from the other slot array and
//      stores it at its own position.
// Stores the unswapped elements would make go to a per-lane dummy word (an exec-mask
// branch per store otherwise). The pivot key P comes from the median in a register.
// xl / xr / dummy: >= kNthWave / 2, kNthWave / 2 and kWave u64 of LDS.
__device__ int64_t nth_step_wave(DGC_LDS uint64_t* q, DGC_LDS uint64_t* xl, DGC_LDS uint64_t* xr,
                                 DGC_LDS uint64_t* dummy, int64_t f, int64_t l, uint32_t P, int64_t nth) {
    constexpr int kTiles = kNthWave / 256 + 1;   // the range <= kNthWave, from a base <= a0
    K5_WSUB_BEGIN();
    const int lane = threadIdx.x & 63;
    const int64_t a0 = f + 1, base = nth_base(q, a0);
    const int nt = (int)uniform32((uint32_t)((l - base + 255) / 256));
    const uint32_t rb0 = (uint32_t)(base - f);   // 0 or 1: tile positions relative to f
    uint64_t x[kTiles][4];
    uint32_t pl[kTiles], pr[kTiles];
#pragma unroll
    for (int u = 0; u < kTiles; ++u) {
        if (u >= nt) break;   // uniform: most tail steps span one or two tiles
        uint32_t valid = 0;
        nth_load4(q, base + 256 * u + 4 * lane, a0, l, x[u], valid);
        stopper_masks(x[u], valid, P, pl[u], pr[u]);
    }
    // per tile: the lane's L / R bases and the tile totals (wave-uniform)
    uint32_t lb[kTiles], rb[kTiles], tl[kTiles], tr[kTiles], TR = 0;
#pragma unroll
    for (int u = 0; u < kTiles; ++u) {
        if (u >= nt) break;
        wave_prefix4(pl[u], lb[u], tl[u]);
        wave_prefix4(pr[u], rb[u], tr[u]);
        TR += tr[u];
    }
    uint32_t runl = 0, runr = 0, nsw = 0, lnext = UINT32_MAX, rmin = UINT32_MAX;
    uint32_t slot[kTiles][4], sw[kTiles];
#pragma unroll
    for (int u = 0; u < kTiles; ++u) {
        if (u >= nt) break;
        uint32_t rl = runl + lb[u], rr = runr + rb[u], bits = 0;
        const uint32_t rel0 = rb0 + 256u * (uint32_t)u + 4u * (uint32_t)lane;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool isl = (pl[u] >> j) & 1u, isr = (pr[u] >> j) & 1u;
            const uint32_t rr_incl = rr + (isr ? 1u : 0u);
            const uint32_t ur = TR - rr_incl;   // right stoppers after this element
            const bool swl = isl && ur >= rl + 1;
            const bool swr = isr && rl >= ur + 1;
            slot[u][j] = swl ? rl : ur;
            *(swl ? xl + rl : swr ? xr + ur : dummy + lane) = x[u][j];
            bits |= (swl ? 1u : 0u) << j | (swr ? 16u : 0u) << j;
            nsw += swl ? 1u : 0u;
            const uint32_t i = rel0 + (uint32_t)j;
            if (isl && !swl && i < lnext) lnext = i;
            if (swr && i < rmin) rmin = i;
            rl += isl ? 1u : 0u;
            rr = rr_incl;
        }
        sw[u] = bits;
        runl += tl[u];
        runr += tr[u];
    }
    const uint32_t s = uniform32(wave_sum(nsw));
    lnext = uniform32(wave_min_u32(lnext));
    rmin = uniform32(wave_min_u32(rmin));
    const int64_t rs = s ? f + (int64_t)rmin : l;
    const int64_t ln = lnext == UINT32_MAX ? INT64_MAX : f + (int64_t)lnext;
    const int64_t cut = ln < rs ? ln : rs;
    // going on left of the cut: the swapped right stoppers (all >= cut) are never read again
    const uint32_t keep = cut > nth ? 0x0Fu : 0xFFu;
    wave_sync();   // the pair slots are written
    K5_WSUB(5);
    uint64_t y[kTiles][4];
#pragma unroll
    for (int u = 0; u < kTiles; ++u) {
        if (u >= nt) break;
        sw[u] &= keep;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool swl = (sw[u] >> j) & 1u, swr = (sw[u] >> (4 + j)) & 1u;
            y[u][j] = *(swl ? xr + slot[u][j] : swr ? xl + slot[u][j] : dummy + lane);
        }
    }
#pragma unroll
    for (int u = 0; u < kTiles; ++u) {
        if (u >= nt) break;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool on = (sw[u] >> j) & 0x11u;
            const uint32_t i = rb0 + 256u * (uint32_t)u + 4u * (uint32_t)lane + (uint32_t)j;
            *(on ? q + f + i : dummy + lane) = y[u][j];
        }
    }
    wave_sync();   // the swaps are done
    K5_WSUB(6);
    return cut;
}

// ---------------------------------------------------------------- register tail
// The last steps (range <= 64 entries): entry i of the range in lane i's registers, so
// a step is ballots, mbcnt and one cross-lane move — no LDS round trip at all. The
// median of three comes from readlanes; L_t's partner is the R stopper with t right
// stoppers after it, i.e. bit TR-1-t of the right-stopper ballot, R's partner with u
// right stoppers after it is bit u of the left-stopper ballot (select_bit).
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)lane);
    return ((uint64_t)hi << 32) | lo;
}

// Position of the k-th (0-based) set bit of m (k < popcount(m)).
__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t k) {
    uint32_t pos = 0, c = (uint32_t)__popc((uint32_t)m);
    uint32_t w = (uint32_t)m;
    if (k >= c) {
        k -= c;
        w = (uint32_t)(m >> 32);
        pos = 32;
    }
#pragma unroll
    for (int b = 16; b >= 1; b >>= 1) {
        c = (uint32_t)__popc(w & ((1u << b) - 1u));
        if (k >= c) {
            k -= c;
            w >>= b;
            pos += (uint32_t)b;
        }
    }
    return pos;
}

// Range q[f, l) of <= 64 entries; returns after the entries are back in q and the
// final insertion sort ran; depth as in nth_tail_wave.
__device__ __forceinline__ void nth_tail_regs(DGC_LDS uint64_t* q, int64_t f, int64_t l, int64_t depth, int64_t nth) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t n = (uint32_t)(l - f);
    uint64_t x = lane < n ? q[f + lane] : 0ull;
    uint32_t F = 0, Lr = n;
    const int64_t nr = nth - f;
    bool heap = false;
    while (Lr - F > 3) {
        if (depth == 0) {
            heap = true;
            break;
        }
        depth -= 1;
        K5_STEP(2);
        // std::__move_median_to_first(F, F+1, mid, Lr-1), as nth_median
        const uint32_t a = F + 1, b = F + (Lr - F) / 2, c = Lr - 1;
        const uint64_t ea = readlane64(x, a), eb = readlane64(x, b), ec = readlane64(x, c), ef = readlane64(x, F);
        const uint32_t ka = qkey(ea), kb = qkey(eb), kc = qkey(ec);
        uint32_t m;
        uint64_t em;
        if (ka > kb) {
            if (kb > kc) { m = b; em = eb; }
            else if (ka > kc) { m = c; em = ec; }
            else { m = a; em = ea; }
        } else if (ka > kc) { m = a; em = ea; }
        else if (kb > kc) { m = c; em = ec; }
        else { m = b; em = eb; }
        x = lane == F ? em : lane == m ? ef : x;
        const uint32_t P = qkey(em);
        // the Hoare partition of [F+1, Lr) around P (nth_step_wave's tests)
        const bool inr = lane > F && lane < Lr;
        const bool isl = inr && qkey(x) <= P, isr = inr && qkey(x) >= P;
        const uint64_t BL = __ballot(isl), BR = __ballot(isr);
        const uint32_t TR = (uint32_t)__popcll(BR);
        const uint32_t rl = mbcnt64(BL, 0u);
        const uint32_t ur = TR - (mbcnt64(BR, 0u) + (isr ? 1u : 0u));
        const bool swl = isl && ur >= rl + 1;
        const bool swr = isr && rl >= ur + 1;
        const uint32_t src = swl ? select_bit(BR, TR - 1u - rl) : swr ? select_bit(BL, ur) : lane;
        const uint64_t y = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(x >> 32), (int)src) << 32) |
                           (uint32_t)__shfl((int)(uint32_t)x, (int)src);
        const uint64_t msl = __ballot(swl), mln = __ballot(isl && !swl), msr = __ballot(swr);
        x = (swl || swr) ? y : x;
        const uint32_t s = (uint32_t)__popcll(msl);
        const uint32_t ln = mln ? (uint32_t)__builtin_ctzll(mln) : 0xFFFFFFFFu;
        const uint32_t rs = s ? (uint32_t)__builtin_ctzll(msr) : Lr;
        const uint32_t cut = ln < rs ? ln : rs;
        if ((int64_t)cut <= nr)
            F = cut;
        else
            Lr = cut;
    }
    if (lane < n) q[f + lane] = x;
    wave_sync();
    if (heap) {
        if (lane == 0) nth_heap_select(q + f + F, nth + 1 - (f + F), (int64_t)(Lr - F), nth - (f + F));
    } else if (lane == 0) {
        nth_insertion_sort(q, f + F, f + Lr);
    }
    wave_sync();
}

// Wave 0 finishes the introselect from sh.f/l/depth (range <= kNthWave, in LDS).
// slots: >= kNthWave + kWave u64 of LDS (the pair slots and the dummy words).
__device__ __forceinline__ void nth_tail_wave(DGC_LDS uint64_t* q, DGC_LDS uint64_t* slots, NthShared& sh, int64_t nth) {
    int64_t f = sh.f, l = sh.l, depth = sh.depth;
    const int lane = threadIdx.x & 63;
    DGC_LDS uint64_t* xl = slots;
    DGC_LDS uint64_t* xr = slots + kNthWave / 2;
    DGC_LDS uint64_t* dummy = slots + kNthWave;
    K5_WSUB_BEGIN();
    while (l - f > 3) {
        if (l - f <= kWave) {   // the rest in registers
            nth_tail_regs(q, f, l, depth, nth);
            return;
        }
        if (depth == 0) {
            if (lane == 0) nth_heap_select(q + f, nth + 1 - f, l - f, nth - f);
            wave_sync();
            return;
        }
        depth -= 1;
        K5_STEP(2);
        K5_WSUB_RESET();
        uint32_t p = 0;
        if (lane == 0) p = nth_median(q, f, l);
        const uint32_t P = uniform32(p);   // lane 0's (every lane is active here)
        wave_sync();
        K5_WSUB(4);
        const int64_t cut = nth_step_wave(q, xl, xr, dummy, f, l, P, nth);
        if (cut <= nth)
            f = cut;
        else
            l = cut;
    }
    if (lane == 0) nth_insertion_sort(q, f, l);
    wave_sync();
}

// ---------------------------------------------------------------- multi-workgroup global phase
// The global-memory steps (range > kNthLds) spread over G workgroups of one tensor
// (k_nth_global, a plain launch sized so that all of them fit at once): one
// workgroup's loads in flight bound the one-workgroup phase (57k candidates: 50 us in
// 2 steps, tools/k5_prof.py). The step is the same partition as nth_step_wg — the G x
// 8 waves take contiguous stretches in order, so every stopper's rank is the same —
// with a barrier among the G workgroups where nth_step_wg has __syncthreads: counts |
// pairing | swaps (+ the advance, run by the last workgroup to arrive).
//
// Residency. A plain launch does not guarantee that the G workgroups run at once (other
// streams' or processes' kernels may hold CUs), and the per-step barriers would then
// wait for a workgroup that cannot start until they exit. So the phase opens with a
// CONSENSUS: every workgroup arrives; the last to arrive votes GO; a workgroup that
// waited kNthGArriveTicks without seeing a vote votes ABORT. The first vote (one CAS on
// `decide`) binds all G workgroups — a late arriver reads ABORT — so either all of them
// are resident and run the phase (resident workgroups stay resident until they exit),
// or none does and k_nth_select replays the whole nth_element on one workgroup from
// [0, n): exact either way, reported as DGC_K5_FALLBACK. A per-step barrier that still
// times out after GO (not expected to happen) marks the run DGC_K5_BROKEN, which the
// engines raise on.
constexpr int kNthGMax = 32;      // workgroups per tensor
constexpr int kNthGMk = 32768;    // stopper bytes per workgroup kept in LDS (512 tiles)
constexpr uint64_t kNthGArriveTicks = 2000000;   // 20 ms of the 100 MHz wall clock
enum : uint32_t { kNthGUndecided = 0, kNthGGo = 1, kNthGAbort = 2 };

struct NthG {
    int64_t f, l, depth;
    unsigned long long l_next, r_min;
    uint32_t pivot, s;
    int32_t heap_exit, go;
    uint32_t bar_count, bar_gen;   // zeroed by k_sel_init, like arrive / decide / status
    uint32_t arrive, decide;       // the residency consensus
    uint32_t status;               // DGC_K5_FALLBACK | DGC_K5_BROKEN of this call
    uint32_t exited;               // workgroups past a GO phase's last barrier (k_nth_select's recovery)
    uint32_t replayed;             // k_nth_select's replay of the tensor done (its extra workgroups emit it)
    uint32_t bl[kNthGMax], br[kNthGMax];
};

// Barrier among the G workgroups of one tensor (all resident: see the consensus above),
// in the form of MI355X_MICROARCH.md's barrier-counter: every wave's stores drained,
// one lane's agent-scope RELEASE fence (the L2 write-back that makes this workgroup's
// stores visible across XCDs), one arrival, a relaxed poll of the generation word with
// s_sleep, one ACQUIRE fence (the L1 invalidate) — two single fences, not the two full
// __threadfence()s per barrier of round 2. The LAST arriver first runs `last` (thread
// 0, after its own acquire: it sees every workgroup's data) and only then releases the
// others, so the step's advance needs no barrier of its own. The spin is bounded
// (~seconds): should it run out, the run is marked DGC_K5_BROKEN instead of hanging.
template <class F>
__device__ __forceinline__ void nthg_barrier(NthG* g, uint32_t G, F&& last) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t gen = __hip_atomic_load(&g->bar_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t a = __hip_atomic_fetch_add(&g->bar_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a == G - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            last();
            __hip_atomic_store(&g->bar_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&g->bar_gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            bool passed = false;
            for (uint32_t spin = 0; spin < (1u << 26); ++spin) {
                if (__hip_atomic_load(&g->bar_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) {
                    passed = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!passed) atomicOr(&g->status, (uint32_t)DGC_K5_BROKEN);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

__device__ __forceinline__ void nthg_barrier(NthG* g, uint32_t G) {
    nthg_barrier(g, G, [] {});
}

// The residency consensus (see above): true = all G workgroups are here, run the phase.
// G_expected is G itself except in the parity tests' forced-fallback mode.
__device__ __forceinline__ bool nthg_consensus(NthG* g, uint32_t G_expected) {
    __shared__ uint32_t verdict;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t a = atomicAdd(&g->arrive, 1u);
        if (a + 1 == G_expected) {
            atomicCAS(&g->decide, (uint32_t)kNthGUndecided, (uint32_t)kNthGGo);
        } else {
            const uint64_t t0 = wall_clock64();
            while (__hip_atomic_load(&g->decide, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == kNthGUndecided) {
                if (wall_clock64() - t0 > kNthGArriveTicks) {
                    atomicCAS(&g->decide, (uint32_t)kNthGUndecided, (uint32_t)kNthGAbort);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        verdict = __hip_atomic_load(&g->decide, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence();
    }
    __syncthreads();
    return verdict == kNthGGo;
}

// Block 0, thread 0: the next step's median and the reset of its results, or the end
// of the phase (go = 0: range <= kNthLds, or the depth-limit heap exit).
__device__ void nthg_prepare(uint64_t* q, NthG* g, int64_t nth) {
    int go = 0;
    if (g->l - g->f > kNthLds && !g->heap_exit) {
        if (g->depth == 0) {
            nth_heap_select(q + g->f, nth + 1 - g->f, g->l - g->f, nth - g->f);
            g->heap_exit = 1;
        } else {
            g->depth -= 1;
            g->pivot = nth_median(q, g->f, g->l);
            g->s = 0;
            g->l_next = ~0ull;
            g->r_min = ~0ull;
            go = 1;
        }
    }
    g->go = go;
}

// The global phase of std::nth_element(q, q + nth, q + n) by G workgroups (block b of
// G); on return g->f / l / depth / heap_exit hold where the one-workgroup kernel goes on.
// Ranges of <= min_run entries are left to the one-workgroup phase: below ~140k
// candidates the four cross-XCD barriers per step cost more than the spread saves
// (tools/k5ab.sh: 100k 0.28 vs 0.25 ms, 500k 0.43 vs 0.94, 1M 0.55 vs 1.44).
// mk: kNthGMk bytes of the caller's LDS (k_nth_select lends the replay's area).
__device__ __forceinline__ void nth_global_multi(uint64_t* q, int64_t n, int64_t nth, uint32_t* lpos, uint32_t* rpos, NthG* g,
                                 uint32_t b, uint32_t G, int64_t min_run, uint32_t G_expected, DGC_LDS uint8_t* mk) {
    constexpr int kB = 8;   // tiles of loads in flight per lane
    __shared__ uint32_t wl[kNthWaves], wr[kNthWaves], pre_l, pre_r, tot_r, s_sh;
    __shared__ int64_t sf, sl;
    __shared__ uint32_t sP;
    __shared__ int sgo;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (n <= min_run || nth >= n) {   // uniform over the G workgroups: no barrier needed
        if (b == 0 && threadIdx.x == 0) {
            g->f = 0;
            g->l = n;
            g->depth = n > 0 ? 2 * (int64_t)(63 - __clzll((unsigned long long)n)) : 0;
            g->heap_exit = 0;
        }
        return;
    }
    if (!nthg_consensus(g, G_expected)) {   // not all resident: one workgroup does it all
        if (b == 0 && threadIdx.x == 0) {
            g->f = 0;
            g->l = n;
            g->depth = n > 0 ? 2 * (int64_t)(63 - __clzll((unsigned long long)n)) : 0;
            g->heap_exit = 0;
            atomicOr(&g->status, (uint32_t)DGC_K5_FALLBACK);
        }
        return;
    }
    if (b == 0 && threadIdx.x == 0) {
        g->f = 0;
        g->l = n;
        g->depth = n > 0 ? 2 * (int64_t)(63 - __clzll((unsigned long long)n)) : 0;
        g->heap_exit = 0;
        if (n > 0 && nth < n)
            nthg_prepare(q, g, nth);
        else
            g->go = 0;
    }
    nthg_barrier(g, G);
    for (;;) {
        if (threadIdx.x == 0) {
            sgo = g->go;
            sf = g->f;
            sl = g->l;
            sP = g->pivot;
        }
        __syncthreads();
        if (!sgo) break;
        const int64_t f = sf, l = sl;
        const uint32_t P = sP;
        const int64_t a0 = f + 1, base = nth_base(q, a0), R = l - base;
        const int64_t GW = (int64_t)G * kNthWaves;
        const int64_t per = ceil_div(ceil_div(R, GW), (int64_t)256) * 256;
        const int64_t bb = base + (int64_t)b * kNthWaves * per;   // this workgroup's first tile
        const int64_t wb = bb + wv * per, we = wb + per < l ? wb + per : l;
        const bool keep = kNthWaves * per / 256 <= kNthGMk / 64;
        // pass 1: stopper counts
        uint32_t cl = 0, cr = 0;
        for (int64_t t0 = wb; t0 < we; t0 += 256 * kB) {
            uint64_t x[kB][4];
            uint32_t valid[kB];
#pragma unroll
            for (int u = 0; u < kB; ++u) nth_load4(q, t0 + u * 256 + 4 * lane, a0, we, x[u], valid[u]);
#pragma unroll
            for (int u = 0; u < kB; ++u) {
                uint32_t pl, pr;
                stopper_masks(x[u], valid[u], P, pl, pr);
                cl += __popc(pl);
                cr += __popc(pr);
                if (keep && t0 + u * 256 < we) mk[((t0 + u * 256 - bb) >> 8) * 64 + lane] = (uint8_t)(pl | (pr << 4));
            }
        }
        cl = wave_sum(cl);
        cr = wave_sum(cr);
        if (lane == 0) {
            wl[wv] = cl;
            wr[wv] = cr;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t a = 0, c = 0;
            for (int i = 0; i < kNthWaves; ++i) {
                a += wl[i];
                c += wr[i];
            }
            g->bl[b] = a;
            g->br[b] = c;
        }
        nthg_barrier(g, G);
        if (threadIdx.x == 0) {
            uint32_t a = 0, c = 0, r = 0;
            for (uint32_t i = 0; i < G; ++i) {
                const uint32_t x = __hip_atomic_load(&g->bl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t y = __hip_atomic_load(&g->br[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a += i < b ? x : 0u;
                r += i < b ? y : 0u;
                c += y;
            }
            pre_l = a;
            pre_r = r;
            tot_r = c;
        }
        __syncthreads();
        // pass 2: ranks, pairing, paired positions; the stoppers before this wave's
        // stretch: the workgroups before b, then the waves before wv
        uint32_t runl = pre_l, runr = pre_r;
        const uint32_t TR = tot_r;
#pragma unroll
        for (int i = 0; i < kNthWaves; ++i) {
            runl += i < wv ? wl[i] : 0u;
            runr += i < wv ? wr[i] : 0u;
        }
        uint32_t paired = 0, lnext = UINT32_MAX, rmin = UINT32_MAX;
        if (keep) {
            for (int64_t t0 = wb; t0 < we; t0 += 256) {
                const uint32_t m = mk[((t0 - bb) >> 8) * 64 + lane];
                pair_tile<false>(m & 15u, m >> 4, t0, f, TR, runl, runr, plain_slots(lpos, rpos), paired, lnext,
                                 rmin);
            }
        } else {
            for (int64_t t0 = wb; t0 < we; t0 += 256 * kB) {
                uint64_t x[kB][4];
                uint32_t valid[kB];
#pragma unroll
                for (int u = 0; u < kB; ++u) nth_load4(q, t0 + u * 256 + 4 * lane, a0, we, x[u], valid[u]);
#pragma unroll
                for (int u = 0; u < kB; ++u) {
                    uint32_t pl, pr;
                    stopper_masks(x[u], valid[u], P, pl, pr);
                    pair_tile<false>(pl, pr, t0 + u * 256, f, TR, runl, runr, plain_slots(lpos, rpos), paired, lnext,
                                     rmin);
                }
            }
        }
        paired = wave_sum(paired);
        lnext = wave_min_u32(lnext);
        rmin = wave_min_u32(rmin);
        if (lane == 0) {
            if (paired) atomicAdd(&g->s, paired);
            if (lnext != UINT32_MAX) atomicMin(&g->l_next, (unsigned long long)(f + lnext));
            if (rmin != UINT32_MAX) atomicMin(&g->r_min, (unsigned long long)(f + rmin));
        }
        nthg_barrier(g, G);
        // pass 3: the swaps L_t <-> R_t, t < s, over all G workgroups (the left halves only
        // when the introselect goes on left of the cut)
        __shared__ int s_left;
        if (threadIdx.x == 0) {
            s_sh = __hip_atomic_load(&g->s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long rm = __hip_atomic_load(&g->r_min, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long ln = __hip_atomic_load(&g->l_next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_left = nth_cut(s_sh, rm, ln, l) > nth;
        }
        __syncthreads();
        nth_swaps<8>(q, plain_slots(lpos, rpos), f, s_sh, b * kNthThreads + threadIdx.x, G * kNthThreads,
                     s_left != 0);
        // the last arriver: the cut, the next range and the next median (all swaps visible)
        nthg_barrier(g, G, [&] {
            const int64_t cut = nth_cut(g->s, g->r_min, g->l_next, g->l);
            if (cut <= nth)
                g->f = cut;
            else
                g->l = cut;
            nthg_prepare(q, g, nth);
        });
    }
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&g->exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// std::nth_element(q, q + nth, q + n, comp) in place, by the calling 512-thread
// workgroup. gpos_l/gpos_r: global pair slots (>= n / 2 + 1 each) for the ranges
// above kNthLds. Returns after a final barrier.
// lq: the caller's LDS area of kNthLds entries (16-B aligned): the partition range
// in the LDS phase, the stopper bytes in the global phase; llp / lrp (kNthPairLds
// each) and lmk (kNthMkLds bytes): the LDS phase's pair slots and stopper bytes.
// from: the state k_nth_global left (its global phase done), or null (start at [0, n)).
__device__ __forceinline__ void nth_element_wg(DGC_GLB uint64_t* q, int64_t n, int64_t nth, DGC_GLB uint32_t* gpos_l,
                                               DGC_GLB uint32_t* gpos_r, DGC_LDS uint64_t* lq, DGC_LDS uint32_t* llp,
                                               DGC_LDS uint32_t* lrp, DGC_LDS uint8_t* lmk,
                                               const NthG* from = nullptr) {
    __shared__ NthShared sh;
    if (threadIdx.x == 0) {
        sh.f = 0;
        sh.l = n;
        sh.depth = n > 0 ? 2 * (int64_t)(63 - __clzll((unsigned long long)n)) : 0;
        sh.heap_exit = 0;
        if (from && n > 0 && nth < n) {
            sh.f = from->f;
            sh.l = from->l;
            sh.depth = from->depth;
            sh.heap_exit = from->heap_exit;
        }
    }
    __syncthreads();
    if (n <= 0 || nth >= n) return;
#ifdef DGC_K5_PROF
    if (threadIdx.x == 0 && blockIdx.x < 64) g_k5prof.bn[blockIdx.x] = n;
#endif
    K5_PROF_BEGIN();
    K5_STAMP(0);
    // global phase: lq (unused until the LDS phase) holds the stopper bytes
    // the whole LDS area (lq, llp, lrp, lmk: contiguous, carved by the caller) is the
    // global phase's arena: stopper bytes + LDS pair slots
    nth_loop_wg<8, 8, true>(q, gpos_l, gpos_r, sh, nth, kNthLds, reinterpret_cast<DGC_LDS uint8_t*>(lq), 0,
                            kNthSmemBytes);
    K5_STAMP(1);
    if (sh.heap_exit) return;
    const int64_t f = sh.f, m = sh.l - sh.f;                          // <= kNthLds entries left
    for (int64_t i = threadIdx.x; i < m; i += kNthThreads) lq[i] = q[f + i];
    __syncthreads();
    if (threadIdx.x == 0) {
        sh.f = 0;
        sh.l = m;
    }
    __syncthreads();
    K5_STAMP(2);
    nth_loop_wg<1, 2, false>(lq, llp, lrp, sh, nth - f, kNthWave, lmk, kNthMkLds / 64);   // LDS phase
    K5_STAMP(3);
    // one wave; its pair slots and dummy words (u64, 8-B aligned) in llp
    static_assert((kNthWave + kWave) * 8 <= kNthPairLds * 4, "tail slots in llp");
    if (!sh.heap_exit && threadIdx.x < kWave)
        nth_tail_wave(lq, reinterpret_cast<DGC_LDS uint64_t*>(llp), sh, nth - f);
    __syncthreads();
    K5_STAMP(4);
    // back to the queue: the positions below k = nth + 1 only (the rest is not output)
    const int64_t mo = nth + 1 - f < m ? nth + 1 - f : m;
    for (int64_t i = threadIdx.x; i < mo; i += kNthThreads) q[f + i] = lq[i];
    __syncthreads();
    K5_STAMP(5);
    K5_PROF_END();
}

}  // namespace dgc
