// 16-bit parameters (bf16 / fp16) on the per-tensor drop-in path.
//
// The reference's memory and compressor run on any float parameter dtype
// (dgc/memory.py:47-48 zeros_like(param), dgc/compression.py:168-177): every ATen op
// on a bf16 / fp16 tensor computes in fp32 and rounds its result to the tensor's
// dtype. Here:
//   K1-16  k_compensate16: momentum correction + velocity accumulation in 16-bit
//          storage, each of the reference's ops rounded to the dtype (round16), and,
//          for the selection, the velocity's exact fp32 image (every bf16 / fp16 value
//          is an fp32 value, order and ties included, so K3 / K4 / K5 run unchanged
//          on it; their threshold *= bound products round to the dtype, thr_dtype);
//   mask   k_mask16: DGCSGDMemory.update's index_fill_ on the 16-bit state;
//   widen  k_widen16: the fp32 image of any 16-bit tensor (a generic memory's output);
//   K6-16  grad.zero_().index_put_(accumulate=True) then mul_(1/W) in the dtype: the
//          CPU index_put_ accumulates serially in index order, rounding every add to
//          the dtype, so the runs (ranks) scatter one launch after another in rank
//          order (indices within one rank's payload are distinct, as DGC emits them),
//          then one pass scales.
// HBM: K1-16 moves 10 B/elem (+4 for the image). Not a BASELINE configuration (every
// benched config is fp32). The batch (DGCBatch / DistributedOptimizer(batch=True) on
// 16-bit parameters) runs K1-16 over its flat 16-bit buffers, dgc_batch_select on the
// image, k_mask_packed16 / k_scatter_packed16 from the packed payloads (their counts
// read on the device), k_gather16 for the optimizer's p.grad tensors.
#include "dgc_common.hpp"

namespace dgc {

template <int DT, bool NEST, bool ACC>
__global__ void __launch_bounds__(kBlock)
k_compensate16(const uint16_t* __restrict__ g, uint16_t* __restrict__ mmt, uint16_t* __restrict__ vec,
               uint16_t* __restrict__ out, float* __restrict__ vec32, int64_t n, float mom) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
        const float gv = h16_to_f32<DT>(g[i]);
        float mv = h16_to_f32<DT>(mmt[i]);
        float vv = ACC ? h16_to_f32<DT>(vec[i]) : 0.f, ov = 0.f;
        if (NEST) {   // mmt.add_(grad).mul_(m); vec.add_(mmt).add_(grad) | out = mmt.add(grad)
            mv = round16<DT>(__fadd_rn(mv, gv));
            mv = round16<DT>(__fmul_rn(mv, mom));
            if (ACC) {
                vv = round16<DT>(__fadd_rn(vv, mv));
                vv = round16<DT>(__fadd_rn(vv, gv));
            } else {
                ov = round16<DT>(__fadd_rn(mv, gv));
            }
        } else {      // mmt.mul_(m).add_(grad); vec.add_(mmt) | out = mmt.clone()
            mv = round16<DT>(__fmul_rn(mv, mom));
            mv = round16<DT>(__fadd_rn(mv, gv));
            if (ACC)
                vv = round16<DT>(__fadd_rn(vv, mv));
            else
                ov = mv;
        }
        mmt[i] = f32_to_h16<DT>(mv);
        if (ACC) {
            vec[i] = f32_to_h16<DT>(vv);
            if (vec32) vec32[i] = vv;
        } else {
            out[i] = f32_to_h16<DT>(ov);
        }
    }
}

template <int DT>
__global__ void __launch_bounds__(kBlock) k_widen16(const uint16_t* __restrict__ x, float* __restrict__ y, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        y[i] = h16_to_f32<DT>(x[i]);
}

template <typename I>
__global__ void __launch_bounds__(kBlock)
k_mask16(uint16_t* __restrict__ mmt, uint16_t* __restrict__ vec, const I* __restrict__ idx, int64_t count,
         int64_t n, int32_t* bad) {
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < count; q += (int64_t)gridDim.x * kBlock) {
        int64_t i = (int64_t)idx[q];
        if (i < 0) i += n;   // index_fill_ wraps negative indices
        if (i < 0 || i >= n) {
            raise_flag(bad);
            continue;
        }
        if (mmt) mmt[i] = 0;   // +0 in both dtypes
        vec[i] = 0;
    }
}

__global__ void __launch_bounds__(kBlock) k_zero16(uint16_t* __restrict__ x, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) x[i] = 0;
}

// One run (rank) of the gathered payload: out[i] = DT(out[i] + DT(v)). values.type(vdtype)
// first (dgc/compression.py:186-187): a wire value of another dtype rounds to DT.
template <int DT, int VD, typename I>
__global__ void __launch_bounds__(kBlock)
k_scatter16(const void* __restrict__ values, const I* __restrict__ idx, int64_t begin, int64_t end,
            uint16_t* __restrict__ out, int64_t n, int32_t* bad) {
    for (int64_t q = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; q < end; q += (int64_t)gridDim.x * kBlock) {
        int64_t i = (int64_t)idx[q];
        if (i < 0) i += n;   // index_put_ wraps negative indices
        if (i < 0 || i >= n) {
            raise_flag(bad);
            continue;
        }
        float v;
        if (VD == DGC_F32)
            v = static_cast<const float*>(values)[q];
        else if (VD == DGC_F16)
            v = f16_to_f32(static_cast<const uint16_t*>(values)[q]);
        else
            v = bf16_to_f32(static_cast<const uint16_t*>(values)[q]);
        v = round16<DT>(v);
        out[i] = f32_to_h16<DT>(__fadd_rn(h16_to_f32<DT>(out[i]), v));
    }
}

// Indices stably sorted (duplicates in input order): the first entry of each run of
// equal indices folds the run in order, rounding every add to DT — index_put_'s serial
// accumulation, for input that does not come as distinct-index runs.
template <int DT, int VD, typename I>
__global__ void __launch_bounds__(kBlock)
k_segsum16(const void* __restrict__ values, const I* __restrict__ idx, int64_t total, uint16_t* __restrict__ out,
           int64_t n, int32_t* bad) {
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < total; q += (int64_t)gridDim.x * kBlock) {
        const int64_t i0 = (int64_t)idx[q];
        if (q > 0 && (int64_t)idx[q - 1] == i0) continue;   // not the first of its run
        int64_t i = i0 < 0 ? i0 + n : i0;
        if (i < 0 || i >= n) {
            raise_flag(bad);
            continue;
        }
        float acc = 0.f;   // grad.zero_()
        for (int64_t e = q; e < total && (int64_t)idx[e] == i0; ++e) {
            float v;
            if (VD == DGC_F32)
                v = static_cast<const float*>(values)[e];
            else if (VD == DGC_F16)
                v = f16_to_f32(static_cast<const uint16_t*>(values)[e]);
            else
                v = bf16_to_f32(static_cast<const uint16_t*>(values)[e]);
            acc = round16<DT>(__fadd_rn(acc, round16<DT>(v)));
        }
        out[i] = f32_to_h16<DT>(acc);
    }
}

template <int DT>
__global__ void __launch_bounds__(kBlock) k_scale16(uint16_t* __restrict__ x, int64_t n, float scale) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
        x[i] = f32_to_h16<DT>(__fmul_rn(h16_to_f32<DT>(x[i]), scale));
}

// ---- the 16-bit batch (dgc_batch_desc.dtype): packed payloads, device counts ----
int64_t payload_layout(int64_t capacity, int vd, int id, int64_t* voff, int64_t* ioff);   // decompress.hip

// DGCSGDMemory.update of one packed payload's entries (its count in the header).
template <typename I>
__global__ void __launch_bounds__(kBlock)
k_mask_packed16(const char* __restrict__ payload, int64_t ioff, uint16_t* __restrict__ mmt,
                uint16_t* __restrict__ vec, int64_t n) {
    const int64_t count = *reinterpret_cast<const int64_t*>(payload);
    const I* idx = reinterpret_cast<const I*>(payload + ioff);
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < count; q += (int64_t)gridDim.x * kBlock) {
        const int64_t i = (int64_t)idx[q];
        if (i < 0 || i >= n) continue;   // our own payload: never out of range
        if (mmt) mmt[i] = 0;
        vec[i] = 0;
    }
}

// One rank's run of a packed payload: out[i] = DT(out[i] + DT(v)) (k_scatter16 with the
// run's count read on the device).
template <int DT, int VD, typename I>
__global__ void __launch_bounds__(kBlock)
k_scatter_packed16(const char* __restrict__ run, int64_t capacity, int64_t voff, int64_t ioff,
                   uint16_t* __restrict__ out, int64_t n, int32_t* bad) {
    int64_t count = *reinterpret_cast<const int64_t*>(run);
    if (count < 0 || count > capacity) {   // a corrupted header: flag it (2), scatter none of it
        if (blockIdx.x == 0 && threadIdx.x == 0) raise_flag(bad, 2);
        count = 0;
    }
    const I* idx = reinterpret_cast<const I*>(run + ioff);
    const void* values = run + voff;
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < count; q += (int64_t)gridDim.x * kBlock) {
        const int64_t i = (int64_t)idx[q];
        if (i < 0 || i >= n) {
            raise_flag(bad);
            continue;
        }
        float v;
        if (VD == DGC_F32)
            v = static_cast<const float*>(values)[q];
        else if (VD == DGC_F16)
            v = f16_to_f32(static_cast<const uint16_t*>(values)[q]);
        else
            v = bf16_to_f32(static_cast<const uint16_t*>(values)[q]);
        v = round16<DT>(v);
        out[i] = f32_to_h16<DT>(__fadd_rn(h16_to_f32<DT>(out[i]), v));
    }
}

// 2-byte multi-tensor gather (the 16-bit gradients into the batch's flat buffer).
constexpr int kG16Max = 64;
struct G16Chunk {
    int32_t count, pad;
    int32_t bstart[kG16Max + 1];
    const uint16_t* src[kG16Max];
    int64_t n[kG16Max];
    int64_t off[kG16Max];
};

__global__ void __launch_bounds__(kBlock) k_gather16(G16Chunk c, uint16_t* __restrict__ dst) {
    int lo = 0, hi = c.count - 1;
    const int b = (int)blockIdx.x;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (c.bstart[mid] <= b) lo = mid; else hi = mid - 1;
    }
    const int64_t n = c.n[lo], off = c.off[lo];
    const uint16_t* __restrict__ src = c.src[lo];
    const int64_t e0 = (int64_t)(b - c.bstart[lo]) * kBlock * 4 + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t e = e0 + (int64_t)j * kBlock;
        if (e < n) dst[off + e] = src[e];
    }
}

static bool is16(int32_t dt) { return dt == DGC_BF16 || dt == DGC_F16; }

template <int DT, typename I>
static int segsum16_t(const void* values, int32_t vd, const I* idx, int64_t total, uint16_t* out, int64_t n,
                      int32_t* bad, hipStream_t s) {
    if (total <= 0) return DGC_OK;
    const int grid = grid_for(total);
    if (vd == DGC_F32)
        hipLaunchKernelGGL((k_segsum16<DT, DGC_F32, I>), dim3(grid), dim3(kBlock), 0, s, values, idx, total, out, n, bad);
    else if (vd == DGC_F16)
        hipLaunchKernelGGL((k_segsum16<DT, DGC_F16, I>), dim3(grid), dim3(kBlock), 0, s, values, idx, total, out, n, bad);
    else
        hipLaunchKernelGGL((k_segsum16<DT, DGC_BF16, I>), dim3(grid), dim3(kBlock), 0, s, values, idx, total, out, n, bad);
    DGC_LAUNCHED();
    return DGC_OK;
}

template <int DT>
static int compensate16_t(const uint16_t* g, uint16_t* m, uint16_t* v, uint16_t* o, float* v32, int64_t n,
                          float mom, bool nest, bool acc, hipStream_t s) {
    const int grid = grid_for(n);
    if (nest && acc)
        hipLaunchKernelGGL((k_compensate16<DT, true, true>), dim3(grid), dim3(kBlock), 0, s, g, m, v, o, v32, n, mom);
    else if (nest)
        hipLaunchKernelGGL((k_compensate16<DT, true, false>), dim3(grid), dim3(kBlock), 0, s, g, m, v, o, v32, n, mom);
    else if (acc)
        hipLaunchKernelGGL((k_compensate16<DT, false, true>), dim3(grid), dim3(kBlock), 0, s, g, m, v, o, v32, n, mom);
    else
        hipLaunchKernelGGL((k_compensate16<DT, false, false>), dim3(grid), dim3(kBlock), 0, s, g, m, v, o, v32, n, mom);
    DGC_LAUNCHED();
    return DGC_OK;
}

template <int DT, typename I>
static int scatter16_t(const void* values, int32_t vd, const I* idx, const int64_t* offs, int32_t nruns,
                       uint16_t* out, int64_t n, int32_t* bad, hipStream_t s) {
    for (int32_t r = 0; r < nruns; ++r) {   // rank order: one launch per run
        const int64_t b = offs[r], e = offs[r + 1];
        if (e <= b) continue;
        const int grid = grid_for(e - b);
        if (vd == DGC_F32)
            hipLaunchKernelGGL((k_scatter16<DT, DGC_F32, I>), dim3(grid), dim3(kBlock), 0, s, values, idx, b, e, out, n, bad);
        else if (vd == DGC_F16)
            hipLaunchKernelGGL((k_scatter16<DT, DGC_F16, I>), dim3(grid), dim3(kBlock), 0, s, values, idx, b, e, out, n, bad);
        else
            hipLaunchKernelGGL((k_scatter16<DT, DGC_BF16, I>), dim3(grid), dim3(kBlock), 0, s, values, idx, b, e, out, n, bad);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

}  // namespace dgc

extern "C" int dgc_compensate16(const void* grad, void* mmt, void* vec, void* out, float* vec32, int64_t n,
                                float momentum, int32_t nesterov, int32_t accumulate, int32_t dtype, void* stream) {
    using namespace dgc;
    if (!is16(dtype)) DGC_FAIL(DGC_ERR_DTYPE, "dgc_compensate16: dtype must be DGC_BF16 or DGC_F16");
    if (n < 0) DGC_FAIL(DGC_ERR_INVALID, "dgc_compensate16: n < 0");
    if (n == 0) return DGC_OK;
    if (!grad || !mmt) DGC_FAIL(DGC_ERR_INVALID, "dgc_compensate16: null grad/mmt");
    if (accumulate && !vec) DGC_FAIL(DGC_ERR_INVALID, "dgc_compensate16: accumulate needs vec");
    if (!accumulate && !out) DGC_FAIL(DGC_ERR_INVALID, "dgc_compensate16: dense branch needs out");
    auto g = static_cast<const uint16_t*>(grad);
    auto m = static_cast<uint16_t*>(mmt);
    auto v = static_cast<uint16_t*>(vec);
    auto o = static_cast<uint16_t*>(out);
    hipStream_t s = static_cast<hipStream_t>(stream);
    return dtype == DGC_BF16 ? compensate16_t<DGC_BF16>(g, m, v, o, vec32, n, momentum, nesterov != 0, accumulate != 0, s)
                             : compensate16_t<DGC_F16>(g, m, v, o, vec32, n, momentum, nesterov != 0, accumulate != 0, s);
}

extern "C" int dgc_widen16(const void* x, float* y, int64_t n, int32_t dtype, void* stream) {
    using namespace dgc;
    if (!is16(dtype)) DGC_FAIL(DGC_ERR_DTYPE, "dgc_widen16: dtype must be DGC_BF16 or DGC_F16");
    if (n < 0 || (n > 0 && (!x || !y))) DGC_FAIL(DGC_ERR_INVALID, "dgc_widen16: bad arguments");
    if (n == 0) return DGC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dtype == DGC_BF16)
        hipLaunchKernelGGL(k_widen16<DGC_BF16>, dim3(grid_for(n)), dim3(kBlock), 0, s, static_cast<const uint16_t*>(x), y, n);
    else
        hipLaunchKernelGGL(k_widen16<DGC_F16>, dim3(grid_for(n)), dim3(kBlock), 0, s, static_cast<const uint16_t*>(x), y, n);
    DGC_LAUNCHED();
    return DGC_OK;
}

extern "C" int dgc_mask_indices16(void* mmt, void* vec, int64_t n, const void* indices, int32_t idtype, int64_t count,
                                  int32_t* bad_flag, void* stream) {
    using namespace dgc;
    if (!vec || (count > 0 && !indices) || !bad_flag) DGC_FAIL(DGC_ERR_INVALID, "dgc_mask_indices16: null argument");
    if (idtype != DGC_I64 && idtype != DGC_I32) DGC_FAIL(DGC_ERR_DTYPE, "dgc_mask_indices16: index dtype");
    if (count <= 0) return DGC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto m = static_cast<uint16_t*>(mmt);
    auto v = static_cast<uint16_t*>(vec);
    if (idtype == DGC_I32)
        hipLaunchKernelGGL(k_mask16<int32_t>, dim3(grid_for(count)), dim3(kBlock), 0, s, m, v,
                           static_cast<const int32_t*>(indices), count, n, bad_flag);
    else
        hipLaunchKernelGGL(k_mask16<int64_t>, dim3(grid_for(count)), dim3(kBlock), 0, s, m, v,
                           static_cast<const int64_t*>(indices), count, n, bad_flag);
    DGC_LAUNCHED();
    return DGC_OK;
}

extern "C" int dgc_decompress16(const void* values, int32_t vdtype, const void* indices, int32_t idtype,
                                const int64_t* run_offsets, int32_t nruns, void* grad, int32_t dtype, int64_t n,
                                float scale, int32_t* bad_flag, void* stream) {
    using namespace dgc;
    if (!is16(dtype)) DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress16: grad dtype must be DGC_BF16 or DGC_F16");
    if (vdtype != DGC_F32 && vdtype != DGC_F16 && vdtype != DGC_BF16)
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress16: value dtype");
    if (idtype != DGC_I64 && idtype != DGC_I32) DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress16: index dtype");
    const bool sorted = nruns == -1;   // one stably index-sorted run: run_offsets = {0, total}
    if (sorted) nruns = 1;
    if (!grad || n < 0 || nruns < 0 || (nruns > 0 && !run_offsets) || !bad_flag)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress16: bad arguments");
    for (int32_t r = 0; r < nruns; ++r)
        if (run_offsets[r + 1] < run_offsets[r] || run_offsets[r] < 0)
            DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress16: run offsets must ascend");
    if (nruns > 0 && run_offsets[nruns] > 0 && (!values || !indices))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress16: null values/indices");
    if (n == 0) return DGC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto out = static_cast<uint16_t*>(grad);
    hipLaunchKernelGGL(k_zero16, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n);   // grad.zero_()
    DGC_LAUNCHED();
    if (sorted) {
        const int64_t total = run_offsets[1] - run_offsets[0];
        const char* vb = static_cast<const char*>(values) + run_offsets[0] * (vdtype == DGC_F32 ? 4 : 2);
        const char* ib = static_cast<const char*>(indices) + run_offsets[0] * (idtype == DGC_I32 ? 4 : 8);
        if (dtype == DGC_BF16 && idtype == DGC_I32)
            DGC_TRY(segsum16_t<DGC_BF16>(vb, vdtype, reinterpret_cast<const int32_t*>(ib), total, out, n, bad_flag, s));
        else if (dtype == DGC_BF16)
            DGC_TRY(segsum16_t<DGC_BF16>(vb, vdtype, reinterpret_cast<const int64_t*>(ib), total, out, n, bad_flag, s));
        else if (idtype == DGC_I32)
            DGC_TRY(segsum16_t<DGC_F16>(vb, vdtype, reinterpret_cast<const int32_t*>(ib), total, out, n, bad_flag, s));
        else
            DGC_TRY(segsum16_t<DGC_F16>(vb, vdtype, reinterpret_cast<const int64_t*>(ib), total, out, n, bad_flag, s));
    } else if (dtype == DGC_BF16) {
        if (idtype == DGC_I32)
            DGC_TRY(scatter16_t<DGC_BF16>(values, vdtype, static_cast<const int32_t*>(indices), run_offsets, nruns, out, n, bad_flag, s));
        else
            DGC_TRY(scatter16_t<DGC_BF16>(values, vdtype, static_cast<const int64_t*>(indices), run_offsets, nruns, out, n, bad_flag, s));
    } else {
        if (idtype == DGC_I32)
            DGC_TRY(scatter16_t<DGC_F16>(values, vdtype, static_cast<const int32_t*>(indices), run_offsets, nruns, out, n, bad_flag, s));
        else
            DGC_TRY(scatter16_t<DGC_F16>(values, vdtype, static_cast<const int64_t*>(indices), run_offsets, nruns, out, n, bad_flag, s));
    }
    if (scale != 1.0f) {   // grad.mul_(1 / W); x 1.0 is the identity in every dtype
        if (dtype == DGC_BF16)
            hipLaunchKernelGGL(k_scale16<DGC_BF16>, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n, scale);
        else
            hipLaunchKernelGGL(k_scale16<DGC_F16>, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n, scale);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

extern "C" int dgc_mask_packed16(const void* payload, int64_t capacity, int32_t vdtype, int32_t idtype, void* mmt,
                                 void* vec, int64_t n, void* stream) {
    using namespace dgc;
    if (!payload || !vec || capacity < 0 || n < 0) DGC_FAIL(DGC_ERR_INVALID, "dgc_mask_packed16: bad arguments");
    if (idtype != DGC_I64 && idtype != DGC_I32) DGC_FAIL(DGC_ERR_DTYPE, "dgc_mask_packed16: index dtype");
    if (capacity == 0) return DGC_OK;
    int64_t voff = 0, ioff = 0;
    payload_layout(capacity, vdtype, idtype, &voff, &ioff);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int grid = grid_for(capacity);
    auto p = static_cast<const char*>(payload);
    auto m = static_cast<uint16_t*>(mmt);
    auto v = static_cast<uint16_t*>(vec);
    if (idtype == DGC_I32)
        hipLaunchKernelGGL(k_mask_packed16<int32_t>, dim3(grid), dim3(kBlock), 0, s, p, ioff, m, v, n);
    else
        hipLaunchKernelGGL(k_mask_packed16<int64_t>, dim3(grid), dim3(kBlock), 0, s, p, ioff, m, v, n);
    DGC_LAUNCHED();
    return DGC_OK;
}

namespace dgc {
template <int DT, typename I>
static int scatter_packed16_t(const char* p, int32_t world, int64_t stride, int64_t capacity, int32_t vd, int64_t voff,
                              int64_t ioff, uint16_t* out, int64_t n, int32_t* bad, hipStream_t s) {
    const int grid = grid_for(capacity);
    for (int32_t r = 0; r < world; ++r) {   // rank order: one launch per run
        const char* run = p + (int64_t)r * stride;
        if (vd == DGC_F32)
            hipLaunchKernelGGL((k_scatter_packed16<DT, DGC_F32, I>), dim3(grid), dim3(kBlock), 0, s, run, capacity, voff, ioff, out, n, bad);
        else if (vd == DGC_F16)
            hipLaunchKernelGGL((k_scatter_packed16<DT, DGC_F16, I>), dim3(grid), dim3(kBlock), 0, s, run, capacity, voff, ioff, out, n, bad);
        else
            hipLaunchKernelGGL((k_scatter_packed16<DT, DGC_BF16, I>), dim3(grid), dim3(kBlock), 0, s, run, capacity, voff, ioff, out, n, bad);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}
}  // namespace dgc

extern "C" int dgc_decompress_packed16(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity,
                                       int32_t vdtype, int32_t idtype, void* grad, int32_t dtype, int64_t n,
                                       float scale, int32_t* bad_flag, void* stream) {
    using namespace dgc;
    if (!is16(dtype)) DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress_packed16: grad dtype must be DGC_BF16 or DGC_F16");
    if (vdtype != DGC_F32 && vdtype != DGC_F16 && vdtype != DGC_BF16)
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress_packed16: value dtype");
    if (idtype != DGC_I64 && idtype != DGC_I32) DGC_FAIL(DGC_ERR_DTYPE, "dgc_decompress_packed16: index dtype");
    if (!payload || !grad || !bad_flag || world < 1 || capacity < 0 || n < 0)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_packed16: bad arguments");
    int64_t voff = 0, ioff = 0;
    const int64_t min_stride = payload_layout(capacity, vdtype, idtype, &voff, &ioff);
    if (rank_stride < min_stride) DGC_FAIL(DGC_ERR_INVALID, "dgc_decompress_packed16: rank_stride < %lld",
                                           (long long)min_stride);
    if (n == 0) return DGC_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto out = static_cast<uint16_t*>(grad);
    hipLaunchKernelGGL(k_zero16, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n);   // grad.zero_()
    DGC_LAUNCHED();
    auto p = static_cast<const char*>(payload);
    if (capacity > 0) {
        if (dtype == DGC_BF16 && idtype == DGC_I32)
            DGC_TRY((scatter_packed16_t<DGC_BF16, int32_t>(p, world, rank_stride, capacity, vdtype, voff, ioff, out, n, bad_flag, s)));
        else if (dtype == DGC_BF16)
            DGC_TRY((scatter_packed16_t<DGC_BF16, int64_t>(p, world, rank_stride, capacity, vdtype, voff, ioff, out, n, bad_flag, s)));
        else if (idtype == DGC_I32)
            DGC_TRY((scatter_packed16_t<DGC_F16, int32_t>(p, world, rank_stride, capacity, vdtype, voff, ioff, out, n, bad_flag, s)));
        else
            DGC_TRY((scatter_packed16_t<DGC_F16, int64_t>(p, world, rank_stride, capacity, vdtype, voff, ioff, out, n, bad_flag, s)));
    }
    if (scale != 1.0f) {   // grad.mul_(1 / W), rounded to the dtype
        if (dtype == DGC_BF16)
            hipLaunchKernelGGL(k_scale16<DGC_BF16>, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n, scale);
        else
            hipLaunchKernelGGL(k_scale16<DGC_F16>, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n, scale);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

extern "C" int dgc_gather16(const void* const* srcs, const int64_t* numels, const int64_t* offsets, int32_t count,
                            void* dst, void* stream) {
    using namespace dgc;
    if (count < 0 || (count > 0 && (!srcs || !numels || !offsets || !dst)))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_gather16: null argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int32_t t0 = 0; t0 < count; t0 += kG16Max) {
        G16Chunk c{};
        c.count = count - t0 < kG16Max ? count - t0 : kG16Max;
        int64_t blocks = 0;
        for (int i = 0; i < c.count; ++i) {
            const int64_t n = numels[t0 + i];
            if (n < 0 || offsets[t0 + i] < 0 || (n > 0 && !srcs[t0 + i]))
                DGC_FAIL(DGC_ERR_INVALID, "dgc_gather16: tensor %d: bad pointer, size or offset", t0 + i);
            c.bstart[i] = (int32_t)blocks;
            c.src[i] = static_cast<const uint16_t*>(srcs[t0 + i]);
            c.n[i] = n;
            c.off[i] = offsets[t0 + i];
            blocks += ceil_div(n, (int64_t)kBlock * 4);
            if (blocks > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_gather16: too many elements");
        }
        c.bstart[c.count] = (int32_t)blocks;
        if (blocks == 0) continue;
        hipLaunchKernelGGL(k_gather16, dim3((unsigned)blocks), dim3(kBlock), 0, s, c, static_cast<uint16_t*>(dst));
        DGC_LAUNCHED();
    }
    return DGC_OK;
}
