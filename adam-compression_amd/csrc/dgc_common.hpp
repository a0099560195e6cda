// Shared device/host helpers for libdgc_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "dgc_hip.h"

namespace dgc {

// ------------------------------------------------------------------ errors
void set_error(const char* fmt, ...);

#define DGC_FAIL(code, ...)            \
    do {                               \
        ::dgc::set_error(__VA_ARGS__); \
        return (code);                 \
    } while (0)

#define DGC_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t _e = (call);                                                        \
        if (_e != hipSuccess)                                                          \
            DGC_FAIL(DGC_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #call,           \
                     hipGetErrorString(_e));                                           \
    } while (0)

#define DGC_LAUNCHED() DGC_HIP(hipGetLastError())

#define DGC_TRY(call)              \
    do {                           \
        int _s = (call);           \
        if (_s != DGC_OK) return _s; \
    } while (0)

// ------------------------------------------------------------------ constants
constexpr int kWave = 64;                 // CDNA wavefront
constexpr int kBlock = 256;               // 4 waves
constexpr int kMaxGrid = 256 * 8;         // 256 CUs x 8 resident 256-thread blocks

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline int grid_for(int64_t work_items, int per_block = kBlock, int cap = kMaxGrid) {
    int64_t g = ceil_div(work_items, per_block);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

__host__ __device__ inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Workspace carving: every region 256-B aligned.
struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(void* b) : base(static_cast<char*>(b)) {}
    template <typename T>
    T* take(size_t count) {
        off = align_up(off, 256);
        T* p = reinterpret_cast<T*>(base ? base + off : nullptr);
        off += count * sizeof(T);
        return p;
    }
    size_t bytes() const { return align_up(off, 256); }
};

// ------------------------------------------------------------------ device helpers
// Workgroups are dispatched round-robin over the 8 XCDs (b % 8), each with its own
// L2. Renumber so every XCD gets a contiguous range of logical blocks: neighbours
// that share cache lines (list boundaries, run bounds, payload lines) then share an
// L2. A bijection on [0, nb) for any nb; speed only, never correctness.
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
    return x * q + (x < r ? x : r) + i;
}

// Address-space-typed pointers. A generic pointer into LDS or global memory becomes a
// flat_ access unless the compiler can prove where it points, and it cannot once two
// stores are merged through a select of their addresses, or a pointer comes out of a
// kernel-argument struct: K5's global-phase loads and pair-slot stores were all flat.
// Typed pointers give ds_ / global_ instructions; as_of<P>::ptr<U> rebinds a pointer
// type to another pointee in the same address space (templates over both kinds).
#define DGC_GLB __attribute__((address_space(1)))
#define DGC_LDS __attribute__((address_space(3)))
template <class P>
struct as_of {
    template <class U>
    using ptr = U*;
};
template <class T>
struct as_of<DGC_GLB T*> {
    template <class U>
    using ptr = DGC_GLB U*;
};
template <class T>
struct as_of<DGC_LDS T*> {
    template <class U>
    using ptr = DGC_LDS U*;
};
template <class P, class U>
using rebind_t = typename as_of<P>::template ptr<U>;
template <class T>
__device__ __forceinline__ DGC_GLB T* glb(T* p) { return (DGC_GLB T*)p; }
template <class T>
__device__ __forceinline__ DGC_LDS T* lds(T* p) { return (DGC_LDS T*)p; }

// Wave-uniform values the compiler cannot prove uniform (threadIdx.x >> 6, LDS reads):
// in SGPRs, loops and branches on them are scalar instead of exec-masked.
__device__ __forceinline__ uint32_t uniform32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t uniform64(int64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int wave_id() { return (int)uniform32(threadIdx.x >> 6); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ uint32_t abs_key(float x) {
    return __float_as_uint(x) & 0x7FFFFFFFu;   // |x| bit pattern: uint order == float order
}

// acc + popcount(m & lanes below this one): two v_mbcnt, no 64-bit mask arithmetic.
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m, uint32_t acc) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, acc));
}

// Exclusive prefix over (lane, j) order of 4 predicate bits per lane (bit j of p),
// i.e. element order 4*lane + j. Returns the lane's base and the wave total.
__device__ __forceinline__ void wave_prefix4(uint32_t p, uint32_t& lane_base, uint32_t& total) {
    const uint64_t m0 = __ballot(p & 1u), m1 = __ballot(p & 2u);
    const uint64_t m2 = __ballot(p & 4u), m3 = __ballot(p & 8u);
    lane_base = mbcnt64(m3, mbcnt64(m2, mbcnt64(m1, mbcnt64(m0, 0u))));
    total = __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
}

__device__ __forceinline__ void wave_prefix1(bool p, uint32_t& lane_base, uint32_t& total) {
    const uint64_t m = __ballot(p);
    lane_base = mbcnt64(m, 0u);
    total = __popcll(m);
}

// ---------------------------------------------------------------- wave64 reductions
// 32-bit reductions and scans over the wave with DPP (gfx9: row_shr within 16-lane
// rows, then row_bcast:15 / row_bcast:31 across rows): VALU ops with a lane-shifted
// operand, a few cycles each, where __shfl_xor / __shfl_up lower to ds_bpermute_b32 —
// an LDS-crossbar round trip each, six dependent ones per reduction, which set the
// pace of every one-wave chain (K5's tail, the last-workgroup steps). Call with all 64
// lanes active. Invalid source lanes (out of the row, or disabled) read `id`.
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_src(uint32_t v, uint32_t id) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)v, CTRL, ROWS, 0xf, false);
}
struct DppAdd {
    static constexpr uint32_t id = 0u;
    __device__ __forceinline__ static uint32_t op(uint32_t a, uint32_t b) { return a + b; }
};
struct DppMax {
    static constexpr uint32_t id = 0u;
    __device__ __forceinline__ static uint32_t op(uint32_t a, uint32_t b) { return a > b ? a : b; }
};
struct DppMin {
    static constexpr uint32_t id = 0xFFFFFFFFu;
    __device__ __forceinline__ static uint32_t op(uint32_t a, uint32_t b) { return a < b ? a : b; }
};
// Inclusive scan in lane order.
template <class Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v = Op::op(v, dpp_src<0x111, 0xf>(v, Op::id));   // row_shr:1
    v = Op::op(v, dpp_src<0x112, 0xf>(v, Op::id));   // row_shr:2
    v = Op::op(v, dpp_src<0x114, 0xf>(v, Op::id));   // row_shr:4
    v = Op::op(v, dpp_src<0x118, 0xf>(v, Op::id));   // row_shr:8
    v = Op::op(v, dpp_src<0x142, 0xa>(v, Op::id));   // row_bcast:15 into rows 1, 3
    v = Op::op(v, dpp_src<0x143, 0xc>(v, Op::id));   // row_bcast:31 into rows 2, 3
    return v;
}
// Whole-wave reduction, wave-uniform (an SGPR).
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan<Op>(v), 63);
}

// 64-bit inclusive add-scan: the same DPP steps on both halves, carry propagated.
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define DGC_SCAN64_STEP(CTRL, ROWS)                                    \
    {                                                                  \
        const uint32_t l2 = dpp_src<CTRL, ROWS>(lo, 0u);               \
        const uint32_t h2 = dpp_src<CTRL, ROWS>(hi, 0u);               \
        const uint32_t nl = lo + l2;                                   \
        hi = hi + h2 + (nl < lo ? 1u : 0u);                            \
        lo = nl;                                                       \
    }
    DGC_SCAN64_STEP(0x111, 0xf)
    DGC_SCAN64_STEP(0x112, 0xf)
    DGC_SCAN64_STEP(0x114, 0xf)
    DGC_SCAN64_STEP(0x118, 0xf)
    DGC_SCAN64_STEP(0x142, 0xa)
    DGC_SCAN64_STEP(0x143, 0xc)
#undef DGC_SCAN64_STEP
    return ((uint64_t)hi << 32) | lo;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    if constexpr (sizeof(T) == 4) {
        return (T)wave_reduce<DppAdd>((uint32_t)v);
    } else {
        const uint64_t s = wave_incl_scan64((uint64_t)v);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)s, 63);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(s >> 32), 63);
        return (T)(((uint64_t)hi << 32) | lo);
    }
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) { return wave_reduce<DppMax>(v); }
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) { return wave_reduce<DppMin>(v); }

// ---------------------------------------------------------------- 16-bit floats
// bf16 <-> fp32 as c10::BFloat16 does it: widening is exact (the 16 bits are the top
// half of the fp32 pattern); narrowing rounds to nearest even, NaN -> 0x7FC0
// (c10/util/BFloat16.h round_to_nearest_even). fp16: v_cvt_f16_f32 (RNE, overflow
// -> inf), as c10::Half.
__host__ __device__ __forceinline__ float bf16_to_f32(uint16_t b) {
    union { uint32_t u; float f; } c{(uint32_t)b << 16};
    return c.f;
}
__host__ __device__ __forceinline__ uint16_t f32_to_bf16(float x) {
    union { float f; uint32_t u; } c{x};
    if ((c.u & 0x7FFFFFFFu) > 0x7F800000u) return (uint16_t)0x7FC0u;
    return (uint16_t)((c.u + 0x7FFFu + ((c.u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
// The empty asm pins x as an fp32 register value: otherwise fptrunc(fmul(fpext(h), m))
// becomes v_fma_mix*_f16 — ONE rounding of the exact product to fp16 where ATen rounds
// the fp32 product first (double rounding; they differ on fp16 ties, e.g. 0.96435546875
// * 0.9f).
__device__ __forceinline__ uint16_t f32_to_f16(float x) {
    asm volatile("" : "+v"(x));
    return __builtin_bit_cast(uint16_t, (_Float16)x);
}
// 16-bit storage of dtype DT (DGC_BF16 / DGC_F16)
template <int DT>
__device__ __forceinline__ float h16_to_f32(uint16_t v) { return DT == DGC_BF16 ? bf16_to_f32(v) : f16_to_f32(v); }
template <int DT>
__device__ __forceinline__ uint16_t f32_to_h16(float x) { return DT == DGC_BF16 ? f32_to_bf16(x) : f32_to_f16(x); }
// fp32 -> DT -> fp32: what one ATen op on a DT tensor leaves (it computes in fp32)
template <int DT>
__device__ __forceinline__ float round16(float x) { return h16_to_f32<DT>(f32_to_h16<DT>(x)); }
// threshold * bound for a tensor of dtype td (0-dim tensor times a Python float: fp32
// product, then rounded to the tensor's dtype)
__device__ __forceinline__ float thr_mul(float t, float f, int td) {
    const float p = __fmul_rn(t, f);
    return td == DGC_BF16 ? round16<DGC_BF16>(p) : td == DGC_F16 ? round16<DGC_F16>(p) : p;
}

// Wire value store (fp32 / fp16 / bf16 round-to-nearest-even, overflow -> inf like torch).
__device__ __forceinline__ void store_value(void* out, int64_t pos, float x, int vdtype) {
    if (vdtype == DGC_BF16)
        reinterpret_cast<uint16_t*>(out)[pos] = f32_to_bf16(x);
    else if (vdtype == DGC_F16)
        reinterpret_cast<__half*>(out)[pos] = __float2half_rn(x);
    else
        reinterpret_cast<float*>(out)[pos] = x;
}

__device__ __forceinline__ void store_index(void* out, int64_t pos, int64_t idx, int idtype) {
    if (idtype == DGC_I32)
        reinterpret_cast<int32_t*>(out)[pos] = (int32_t)idx;
    else
        reinterpret_cast<int64_t*>(out)[pos] = idx;
}

// ---------------------------------------------------------------- block scan
// Exclusive scan of one u64 per thread over the block (blockDim a multiple of 64,
// <= 1024); returns the exclusive prefix and writes the block total to *total.
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* lds16, uint64_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan64(v);
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

}  // namespace dgc

namespace dgc {
// Streaming (non-temporal) 16-B accesses: data touched once per pass bypasses
// cache allocation (measured on MI355X, 1B elements: 3R2W update 5.57 -> 5.86 TB/s,
// read-only 5.98 -> 6.62 TB/s; see tools/membench.hip).
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const f4v x = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
    return make_float4(x[0], x[1], x[2], x[3]);
}

__device__ __forceinline__ void st_nt(float4* p, const float4& v) {
    const f4v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f4v*>(p));
}

// The streaming stores of the big passes (K1's momentum / velocity, the dense zero
// fill), by size. An nt store keeps its line dirty in L2, and the kernel boundary then
// writes the XCD L2s back before the next kernel starts: + dirty bytes / ~6 TB/s
// (MI355X_MICROARCH.md, "boundary"), ~5 us of idle GPU after K1 (8 x 4 MB of L2 full
// of dirty lines). A write-through store (sc1: the line dropped from the XCD's L2)
// leaves nothing behind, but streams ~10 % slower: same box, flat-1B K1 3.75 ms with
// sc1 against 3.42 ms nt, VGG-16-BN 0.54 against 0.48 ms, while ResNet-50's 25.5M
// elements run 0.088 ms sc1 against 0.097 ms nt. So a pass over at most
// kWriteThroughMax elements writes through (wt), a larger one stores nt. The asm store
// ends with s_nop 1: hipcc does not pad an asm statement, and its next instruction
// could otherwise overwrite the data registers before the store has read them
// (cdna_hip_programming.md §5.7 item 1).
constexpr int64_t kWriteThroughMax = 48LL << 20;
inline bool write_through(int64_t elements) { return elements <= kWriteThroughMax; }

__device__ __forceinline__ void st_stream(float4* p, const float4& v, bool wt) {
    if (wt) {   // uniform
        const f4v x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" : : "v"(p), "v"(x) : "memory");
    } else {
        st_nt(p, v);
    }
}
}  // namespace dgc

namespace dgc {
// Strided sample of |vec| fused into K1 (dgc/compression.py:113,119).
struct SampleSpec {
    float* out;        // nullptr: no sampling
    int64_t start;
    int64_t stride;    // >= 4 on the fused path
    int64_t count;     // ceil((n - start) / stride)
    double inv_stride; // 1.0 / stride
    float inv_stride_f;
};

// q = t / s, r = t % s for 4 <= s < 2^23 and t < 2^24: a float-reciprocal estimate
// is within one of the quotient (relative error <= 2^-23, |q error| <= 2/s), then
// one correction step. Larger strides take the integer divide (uniform branch).
__device__ __forceinline__ void divmod_u32(uint32_t t, uint32_t s, float inv, uint32_t& q, uint32_t& r) {
    if (s < (1u << 23)) {
        q = (uint32_t)__fmul_rn((float)t, inv);
        int32_t rr = (int32_t)(t - q * s);
        if (rr < 0) {
            q -= 1;
            rr += (int32_t)s;
        } else if (rr >= (int32_t)s) {
            q += 1;
            rr -= (int32_t)s;
        }
        r = (uint32_t)rr;
    } else {
        q = t / s;
        r = t - q * s;
    }
}

// floor/mod of d by s for |d| < 2^53 without a 64-bit integer divide: a double
// estimate, then an exact integer correction.
__device__ __forceinline__ void floor_divmod_fast(int64_t d, int64_t s, double inv, int64_t& q, int64_t& r) {
    q = (int64_t)floor((double)d * inv);
    r = d - q * s;
    while (r < 0) {
        r += s;
        q -= 1;
    }
    while (r >= s) {
        r -= s;
        q += 1;
    }
}

// DGCSGDMemory.compensate on one element (dgc/memory.py:50-70), every op rounded
// to fp32 like the reference's separate ATen add_/mul_ ops (no FMA contraction):
//   nesterov: m = (m + g) * mom;  v = (v + m) + g      (dense branch: out = m + g)
//   plain:    m = m * mom + g;    v = v + m            (dense branch: out = m)
template <bool NEST, bool ACC>
__device__ __forceinline__ float comp1(float g, float& m, float& v, float mom) {
    if (NEST) {
        m = __fmul_rn(__fadd_rn(m, g), mom);
        if (ACC) {
            v = __fadd_rn(__fadd_rn(v, m), g);
            return v;
        }
        return __fadd_rn(m, g);
    }
    m = __fadd_rn(__fmul_rn(m, mom), g);
    if (ACC) {
        v = __fadd_rn(v, m);
        return v;
    }
    return m;
}
// ---------------------------------------------------------------- error flags
// A flag the host polls without synchronising (an engine's pinned status sink) or a
// device int32: every writer stores the same constant — idempotent, so no
// read-modify-write has to cross PCIe — at system scope, so the store reaches host
// memory and not only this XCD's L2. Written only on an error path.
__device__ __forceinline__ void raise_flag(int32_t* f, int32_t v = 1) {
    if (f) __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------- last arrival
// True in every thread of the workgroup that arrives last at `ticket` among
// `nblocks`. The data handed to the last workgroup is ONLY device-scope atomics
// (histogram / count adds) that it reads back with agent-scope atomic loads — the
// "agent atomics both sides" form of cdna_hip_programming.md G16 — so no L2
// write-back (release) or L1 invalidate (acquire) fence is needed: every wave
// drains its atomics (vmcnt(0): acknowledged = performed at the coherence point)
// before the barrier, then one lane draws the ticket.
__device__ __forceinline__ bool last_block_arrival(uint32_t* ticket, uint32_t nblocks) {
    __shared__ int is_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = t == nblocks - 1;
        if (is_last) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // reusable
    }
    __syncthreads();
    return is_last;
}

// last_block_arrival for many workgroups: arrivals spread over 8 shard counters (lb %
// 8: one shard per XCD under round-robin placement), and the shard's last arrival
// arrives at the top counter tk[8] — a ~1000-way arrival on one word costs ~12 us
// (MI355X_MICROARCH.md "fanin"), eight ~125-way ones run side by side. tk: 9 words,
// zero at rest (each last arrival resets its word). lb: the block's index among the
// nblocks of the task.
__device__ __forceinline__ bool last_block_arrival8(uint32_t* tk, uint32_t lb, uint32_t nblocks) {
    if (nblocks <= 64) return last_block_arrival(tk + 8, nblocks);
    __shared__ int is_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t sh = lb & 7u;
        const uint32_t members = nblocks / 8 + (sh < (nblocks & 7u) ? 1u : 0u);
        const uint32_t a = __hip_atomic_fetch_add(tk + sh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int last = 0;
        if (a == members - 1) {
            __hip_atomic_store(tk + sh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t b = __hip_atomic_fetch_add(tk + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (b == 7u) {
                __hip_atomic_store(tk + 8, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last = 1;
            }
        }
        is_last = last;
    }
    __syncthreads();
    return is_last;
}

// ---------------------------------------------------------------- chained launches
// The end of one phase of a chained launch (k_chain_one, k_rs_passes), by the whole
// workgroup. Its stores are drained into its XCD's L2 and its completed virtual blocks
// added to its XCD's count (done[8]: one word per XCD, so a count > 0 also says the XCD
// holds writes of the phase). Once all nvb blocks are done, ONE workgroup per such XCD
// writes that XCD's L2 back (agent release; `xrel[x]` elects it, `rel` counts them) —
// not every workgroup: each release writes back the whole XCD L2, ~1.7-6.5 us
// (MI355X_MICROARCH.md §inter-workgroup visibility), and a phase of 2048 workgroups paid
// it 2048 times. Then every workgroup acquires (its CU's L1) and goes on. Words zero at
// the start of the call. (The s_waitcnt after the release: the ROCm 7.2 hazard that can
// drop it; after the acquire: its invalidate completes asynchronously.)
struct ChainPhase {
    uint32_t done[8];
    uint32_t rel;
    uint32_t xrel[8];
    uint32_t pad[15];
};
static_assert(sizeof(ChainPhase) == 128, "one 128-B line per phase");

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x & 7u;
}

__device__ __forceinline__ void chain_phase_end(ChainPhase* cp, uint32_t mine, uint32_t nvb) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t x = xcc_id();
        if (mine) __hip_atomic_fetch_add(&cp->done[x], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t m = 0;
        for (;;) {
            uint32_t tot = 0;
            m = 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const uint32_t c = __hip_atomic_load(&cp->done[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                tot += c;
                m |= (c ? 1u : 0u) << i;
            }
            if (tot >= nvb) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (((m >> x) & 1u) && atomicCAS(&cp->xrel[x], 0u, 1u) == 0u) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&cp->rel, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        while (__hip_atomic_load(&cp->rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)__popc(m))
            __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

}  // namespace dgc
