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
//   > kNthLds entries   in global memory (L2 / Infinity-Cache resident), 8 waves, each
//                       over a contiguous stretch, 4 tiles of loads in flight per lane;
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
constexpr int kNthBatch = 4;     // 256-entry tiles loaded per lane before use

__device__ __forceinline__ uint32_t qkey(uint64_t e) { return (uint32_t)(e >> 32); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- heaps (depth limit)
// std::__adjust_heap + std::__push_heap on q[0..n) with comp = key greater (the
// heap's "largest" is the smallest key). Single thread.
__device__ void nth_adjust_heap(uint64_t* q, int64_t hole, int64_t n, uint64_t v) {
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
__device__ void nth_heap_select(uint64_t* q, int64_t mid, int64_t n, int64_t nth) {
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

// std::__move_median_to_first(f, f+1, mid, l-1) with comp = key greater. One thread.
__device__ __forceinline__ void nth_median(uint64_t* q, int64_t f, int64_t l) {
    const int64_t a = f + 1, b = f + (l - f) / 2, c = l - 1;
    const uint32_t ka = qkey(q[a]), kb = qkey(q[b]), kc = qkey(q[c]);
    int64_t m;
    if (ka > kb)
        m = kb > kc ? b : (ka > kc ? c : a);
    else
        m = ka > kc ? a : (kb > kc ? c : b);
    const uint64_t t = q[f];
    q[f] = q[m];
    q[m] = t;
}

// std::__insertion_sort of q[f, l) (<= 3 entries after the loop). One thread.
__device__ void nth_insertion_sort(uint64_t* q, int64_t f, int64_t l) {
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

// Lane's 4 consecutive entries of a 256-entry tile (positions < end).
__device__ __forceinline__ void nth_load4(const uint64_t* q, int64_t e0, int64_t end, uint64_t (&x)[4],
                                          uint32_t& valid) {
    valid = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool ok = e0 + j < end;
        x[j] = ok ? q[e0 + j] : 0ull;
        valid |= (uint32_t)ok << j;
    }
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

// Pass 2 on one tile: ranks, pairing and the paired positions. rl / rr: the left and
// right stoppers before the tile (uniform over the wave); lpos/rpos hold positions
// relative to f. Returns via the accumulators.
__device__ __forceinline__ void pair_tile(const uint64_t (&x)[4], uint32_t valid, uint32_t P, int64_t e0, int64_t f,
                                          uint32_t TR, uint32_t& runl, uint32_t& runr, uint32_t* lpos, uint32_t* rpos,
                                          uint32_t& paired, unsigned long long& lnext, unsigned long long& rmin) {
    uint32_t pl, pr;
    stopper_masks(x, valid, P, pl, pr);
    uint32_t bl, tl, br, tr;
    wave_prefix4(pl, bl, tl);
    wave_prefix4(pr, br, tr);
    uint32_t rl = runl + bl;   // left stoppers before this element
    uint32_t rr = runr + br;   // right stoppers in [f+1, this element)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool isl = (pl >> j) & 1u, isr = (pr >> j) & 1u;
        const int64_t i = e0 + j;
        const uint32_t rr_incl = rr + (isr ? 1u : 0u);
        if (isl) {
            // L_{rl+1} = i is swapped iff #(key >= P in (i, l)) >= rl + 1
            if (TR - rr_incl >= rl + 1) {
                lpos[rl] = (uint32_t)(i - f);
                ++paired;
            } else if ((unsigned long long)i < lnext) {
                lnext = (unsigned long long)i;
            }
        }
        if (isr) {
            // R_{u+1} = i with u = #(key >= P in (i, l)); swapped iff #(key <= P in [f+1, i)) >= u + 1
            const uint32_t u = TR - rr_incl;
            if (rl >= u + 1) {
                rpos[u] = (uint32_t)(i - f);
                if ((unsigned long long)i < rmin) rmin = (unsigned long long)i;
            }
        }
        rl += isl;
        rr = rr_incl;
    }
    runl += tl;
    runr += tr;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long a = __shfl_xor(v, o);
        v = a < v ? a : v;
    }
    return v;
}

// ---------------------------------------------------------------- workgroup step
struct NthShared {
    int64_t f, l, depth;
    uint32_t wl[kNthWaves], wr[kNthWaves];   // per-wave stopper counts
    uint32_t s;                              // swaps
    unsigned long long l_next, r_min;
    int heap_exit;
};

// One partition step over q[f, l) by the whole workgroup; the pivot is already at
// q[f] and sh.s / l_next / r_min are reset. On return (after the last barrier) the
// step's swaps are done and sh.s / l_next / r_min hold its result.
__device__ void nth_step_wg(uint64_t* q, uint32_t* lpos, uint32_t* rpos, NthShared& sh) {
    const int64_t f = sh.f, l = sh.l;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t P = qkey(q[f]);
    const int64_t a0 = f + 1, R = l - a0;
    const int64_t per = ceil_div(ceil_div(R, (int64_t)kNthWaves), (int64_t)256) * 256;
    const int64_t wb = a0 + wv * per, we = wb + per < l ? wb + per : l;
    // pass 1: stopper counts per wave, kNthBatch tiles of loads in flight per lane
    uint32_t cl = 0, cr = 0;
    for (int64_t t0 = wb; t0 < we; t0 += 256 * kNthBatch) {
        uint64_t x[kNthBatch][4];
        uint32_t valid[kNthBatch];
#pragma unroll
        for (int b = 0; b < kNthBatch; ++b) nth_load4(q, t0 + b * 256 + 4 * lane, we, x[b], valid[b]);
#pragma unroll
        for (int b = 0; b < kNthBatch; ++b) {
            uint32_t pl, pr;
            stopper_masks(x[b], valid[b], P, pl, pr);
            cl += __popc(pl);
            cr += __popc(pr);
        }
    }
    cl = wave_sum(cl);
    cr = wave_sum(cr);
    if (lane == 0) {
        sh.wl[wv] = cl;
        sh.wr[wv] = cr;
    }
    __syncthreads();
    // every wave derives its own prefix and the total from the 16 wave counts
    uint32_t runl = 0, runr = 0, TR = 0;
#pragma unroll
    for (int i = 0; i < kNthWaves; ++i) {
        const uint32_t a = sh.wl[i], b = sh.wr[i];
        runl += i < wv ? a : 0u;
        runr += i < wv ? b : 0u;
        TR += b;
    }
    // pass 2: ranks, pairing, paired positions
    uint32_t paired = 0;
    unsigned long long lnext = ~0ull, rmin = ~0ull;
    for (int64_t t0 = wb; t0 < we; t0 += 256 * kNthBatch) {
        uint64_t x[kNthBatch][4];
        uint32_t valid[kNthBatch];
#pragma unroll
        for (int b = 0; b < kNthBatch; ++b) nth_load4(q, t0 + b * 256 + 4 * lane, we, x[b], valid[b]);
#pragma unroll
        for (int b = 0; b < kNthBatch; ++b)
            pair_tile(x[b], valid[b], P, t0 + b * 256 + 4 * lane, f, TR, runl, runr, lpos, rpos, paired, lnext, rmin);
    }
    paired = wave_sum(paired);
    lnext = wave_min_u64(lnext);
    rmin = wave_min_u64(rmin);
    if (lane == 0) {
        if (paired) atomicAdd(&sh.s, paired);
        if (lnext != ~0ull) atomicMin(&sh.l_next, lnext);
        if (rmin != ~0ull) atomicMin(&sh.r_min, rmin);
    }
    __syncthreads();
    // pass 3: the swaps L_t <-> R_t, t < s (disjoint positions)
    const uint32_t s = sh.s;
    for (uint32_t t = threadIdx.x; t < s; t += kNthThreads) {
        const int64_t li = f + lpos[t], ri = f + rpos[t];
        const uint64_t a = q[li], b = q[ri];
        q[li] = b;
        q[ri] = a;
    }
    __syncthreads();
}

// Thread 0, after a step: the cut, the next range, and either the next step's
// median (returns 1), a depth-limit heap exit, or the end of this phase (returns 0).
__device__ int nth_advance(uint64_t* q, NthShared& sh, int64_t nth, int64_t stop) {
    const int64_t rs = sh.s ? (int64_t)sh.r_min : sh.l;
    const int64_t ln = sh.l_next == ~0ull ? INT64_MAX : (int64_t)sh.l_next;
    const int64_t cut = ln < rs ? ln : rs;
    if (cut <= nth)
        sh.f = cut;
    else
        sh.l = cut;
    return 0;
}

// The introselect loop on q[f, l) by the whole workgroup while the range exceeds
// `stop` entries; ends with a barrier, sh.f/l/depth updated or sh.heap_exit set.
__device__ void nth_loop_wg(uint64_t* q, uint32_t* lpos, uint32_t* rpos, NthShared& sh, int64_t nth,
                            int64_t stop) {
    // thread 0 prepares a step: depth check, median, reset of the step's results
    auto prepare = [&]() -> bool {
        if (sh.l - sh.f <= stop) return false;
        if (sh.depth == 0) {
            nth_heap_select(q + sh.f, nth + 1 - sh.f, sh.l - sh.f, nth - sh.f);
            sh.heap_exit = 1;
            return false;
        }
        sh.depth -= 1;
        nth_median(q, sh.f, sh.l);
        sh.s = 0;
        sh.l_next = ~0ull;
        sh.r_min = ~0ull;
        return true;
    };
    __shared__ int go;
    if (threadIdx.x == 0) go = !sh.heap_exit && prepare();
    __syncthreads();
    while (go) {
        nth_step_wg(q, lpos, rpos, sh);
        if (threadIdx.x == 0) {
            nth_advance(q, sh, nth, stop);
            go = prepare();
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- single-wave tail
// The same step by one wave on an LDS range of <= kNthWave entries: no workgroup barrier.
__device__ int64_t nth_step_wave(uint64_t* q, uint32_t* lpos, uint32_t* rpos, int64_t f, int64_t l) {
    const int lane = threadIdx.x & 63;
    const uint32_t P = qkey(q[f]);
    const int64_t a0 = f + 1;
    uint32_t cr = 0;
    for (int64_t t0 = a0; t0 < l; t0 += 256) {
        uint64_t x[4];
        uint32_t valid, pl, pr;
        nth_load4(q, t0 + 4 * lane, l, x, valid);
        stopper_masks(x, valid, P, pl, pr);
        cr += __popc(pr);
    }
    const uint32_t TR = wave_sum(cr);
    uint32_t runl = 0, runr = 0, paired = 0;
    unsigned long long lnext = ~0ull, rmin = ~0ull;
    for (int64_t t0 = a0; t0 < l; t0 += 256) {
        uint64_t x[4];
        uint32_t valid;
        nth_load4(q, t0 + 4 * lane, l, x, valid);
        pair_tile(x, valid, P, t0 + 4 * lane, f, TR, runl, runr, lpos, rpos, paired, lnext, rmin);
    }
    const uint32_t s = wave_sum(paired);
    lnext = wave_min_u64(lnext);
    rmin = wave_min_u64(rmin);
    wave_sync();   // the pair slots are written
    for (uint32_t t = lane; t < s; t += kWave) {
        const int64_t li = f + lpos[t], ri = f + rpos[t];
        const uint64_t a = q[li], b = q[ri];
        q[li] = b;
        q[ri] = a;
    }
    wave_sync();   // the swaps are done
    const int64_t rs = s ? (int64_t)rmin : l;
    const int64_t ln = lnext == ~0ull ? INT64_MAX : (int64_t)lnext;
    return ln < rs ? ln : rs;
}

// Wave 0 finishes the introselect from sh.f/l/depth (range <= kNthWave, in LDS).
__device__ void nth_tail_wave(uint64_t* q, uint32_t* lpos, uint32_t* rpos, NthShared& sh, int64_t nth) {
    int64_t f = sh.f, l = sh.l, depth = sh.depth;
    const int lane = threadIdx.x & 63;
    while (l - f > 3) {
        if (depth == 0) {
            if (lane == 0) nth_heap_select(q + f, nth + 1 - f, l - f, nth - f);
            wave_sync();
            return;
        }
        depth -= 1;
        if (lane == 0) nth_median(q, f, l);
        wave_sync();
        const int64_t cut = nth_step_wave(q, lpos, rpos, f, l);
        if (cut <= nth)
            f = cut;
        else
            l = cut;
    }
    if (lane == 0) nth_insertion_sort(q, f, l);
    wave_sync();
}

// std::nth_element(q, q + nth, q + n, comp) in place, by the calling 512-thread
// workgroup. gpos_l/gpos_r: global pair slots (>= n / 2 + 1 each) for the ranges
// above kNthLds. Returns after a final barrier.
__device__ void nth_element_wg(uint64_t* q, int64_t n, int64_t nth, uint32_t* gpos_l, uint32_t* gpos_r) {
    __shared__ NthShared sh;
    __shared__ uint64_t lq[kNthLds];
    __shared__ uint32_t llp[kNthLds / 2 + 1], lrp[kNthLds / 2 + 1];
    if (threadIdx.x == 0) {
        sh.f = 0;
        sh.l = n;
        sh.depth = n > 0 ? 2 * (int64_t)(63 - __clzll((unsigned long long)n)) : 0;
        sh.heap_exit = 0;
    }
    __syncthreads();
    if (n <= 0 || nth >= n) return;
    nth_loop_wg(q, gpos_l, gpos_r, sh, nth, kNthLds);                 // global phase
    if (sh.heap_exit) return;
    const int64_t f = sh.f, m = sh.l - sh.f;                          // <= kNthLds entries left
    for (int64_t i = threadIdx.x; i < m; i += kNthThreads) lq[i] = q[f + i];
    __syncthreads();
    if (threadIdx.x == 0) {
        sh.f = 0;
        sh.l = m;
    }
    __syncthreads();
    nth_loop_wg(lq, llp, lrp, sh, nth - f, kNthWave);                  // LDS phase, all waves
    if (!sh.heap_exit && threadIdx.x < kWave) nth_tail_wave(lq, llp, lrp, sh, nth - f);   // one wave
    __syncthreads();
    for (int64_t i = threadIdx.x; i < m; i += kNthThreads) q[f + i] = lq[i];
    __syncthreads();
}

}  // namespace dgc
