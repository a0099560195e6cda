// K7: DGCSGD.step fused — weight-decay momentum and the parameter update in one
// streaming pass over every parameter of a group (dgc/optim/sgd.py:42-68).
//
// DGC applies the gradient's momentum in DGCSGDMemory.compensate, so the optimizer
// keeps momentum for the weight-decay term only. Per element, with the reference's
// torch-CPU rounding (probed: Tensor * python-float = fl(x * fl32(s)); add(b, alpha)
// = fmadd(b, alpha, a), ONE rounding, in both the vector and the scalar loops):
//
//   wd != 0:  d = p * wd                                  (mul)
//             mom != 0:  first step:  buf = d             (momentum_buffer = d_p)
//                        else:        buf = buf * mom     (mul_)
//                                     buf = fma(d, 1 - dampening, buf)   (add_(alpha))
//                        nesterov:    d = fma(buf, mom, d)               (add(alpha))
//                        else:        d = buf
//             d = d + g                                   (add)
//   wd == 0:  d = g
//   p = fma(d, -lr, p)                                    (add_(alpha=-lr))
//
// HBM: read p, g (+ buf), write p (+ buf): 12 or 20 B per element. One launch covers
// up to kSgdMaxTensors tensors (a block table in the kernel arguments, like a
// multi-tensor apply); each block streams 16-B vectors of one tensor.
#include "dgc_common.hpp"

namespace dgc {

constexpr int kSgdMaxTensors = 48;
constexpr int kSgdPerBlock = kBlock * 4 * 4;   // 4 float4 per lane per block

struct SgdTable {
    float* p[kSgdMaxTensors];
    const float* g[kSgdMaxTensors];
    float* buf[kSgdMaxTensors];
    int64_t n[kSgdMaxTensors];
    int32_t block0[kSgdMaxTensors + 1];   // first block of each tensor; block0[count] = grid
    int32_t first[kSgdMaxTensors];        // momentum buffer created on this step
    int32_t count;
};

struct SgdHyper {
    float wd, mom, damp_alpha, neg_lr;
    int32_t nesterov;
};

template <bool WD, bool MOM>
__device__ __forceinline__ float sgd1(float p, float g, float& b, bool first, const SgdHyper& h) {
    float d = g;
    if (WD) {
        d = __fmul_rn(p, h.wd);
        if (MOM) {
            if (first) {
                b = d;
            } else {
                b = __fmul_rn(b, h.mom);
                b = __fmaf_rn(d, h.damp_alpha, b);
            }
            d = h.nesterov ? __fmaf_rn(b, h.mom, d) : b;
        }
        d = __fadd_rn(d, g);
    }
    return __fmaf_rn(d, h.neg_lr, p);
}

template <bool WD, bool MOM>
__global__ void __launch_bounds__(kBlock) k_sgd(SgdTable t, SgdHyper h) {
    // the tensor of this block: block0 is ascending, <= 48 entries (scalar search)
    int ti = 0;
    while (ti + 1 < t.count && (int)blockIdx.x >= t.block0[ti + 1]) ++ti;
    float* __restrict__ p = t.p[ti];
    const float* __restrict__ g = t.g[ti];
    float* __restrict__ buf = t.buf[ti];
    const int64_t n = t.n[ti];
    const bool first = t.first[ti] != 0;
    const int64_t base = (int64_t)(blockIdx.x - t.block0[ti]) * kSgdPerBlock;
    const bool vec = aligned16(p) && aligned16(g) && (!MOM || aligned16(buf));
    if (vec && base + kSgdPerBlock <= n) {
        float4 pv[4], gv[4], bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + (int64_t)(u * kBlock + threadIdx.x) * 4;
            pv[u] = ld_nt(reinterpret_cast<const float4*>(p + i));
            gv[u] = ld_nt(reinterpret_cast<const float4*>(g + i));
            if (MOM && !first) bv[u] = ld_nt(reinterpret_cast<const float4*>(buf + i));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + (int64_t)(u * kBlock + threadIdx.x) * 4;
            float4 o;
            o.x = sgd1<WD, MOM>(pv[u].x, gv[u].x, bv[u].x, first, h);
            o.y = sgd1<WD, MOM>(pv[u].y, gv[u].y, bv[u].y, first, h);
            o.z = sgd1<WD, MOM>(pv[u].z, gv[u].z, bv[u].z, first, h);
            o.w = sgd1<WD, MOM>(pv[u].w, gv[u].w, bv[u].w, first, h);
            st_nt(reinterpret_cast<float4*>(p + i), o);
            if (MOM) st_nt(reinterpret_cast<float4*>(buf + i), bv[u]);
        }
        return;
    }
    const int64_t end = base + kSgdPerBlock < n ? base + kSgdPerBlock : n;
    for (int64_t i = base + threadIdx.x; i < end; i += kBlock) {
        float b = MOM && !first ? buf[i] : 0.f;
        p[i] = sgd1<WD, MOM>(p[i], g[i], b, first, h);
        if (MOM) buf[i] = b;
    }
}

// K7-16: DGCSGD.step on bf16 / fp16 parameters (DT): the same op sequence, every ATen
// op rounding to the dtype (it computes in fp32). `x.add(y, alpha)` on a 16-bit CPU
// tensor rounds alpha to the dtype; its vectorised body (the first n - n % 32 elements)
// rounds fl32(x + y * alpha) once (the product of two 16-bit values is exact in fp32),
// its scalar tail rounds the product to the dtype first (oracle.dgcsgd_step16, pinned
// to the reference's run in tests/golden/sgd16.*). 6 or 10 B per element.
constexpr int kSgd16PerThread = 4;
constexpr int kSgd16PerBlock = kBlock * kSgd16PerThread;

struct Sgd16Table {
    uint16_t* p[kSgdMaxTensors];
    const uint16_t* g[kSgdMaxTensors];
    uint16_t* buf[kSgdMaxTensors];
    int64_t n[kSgdMaxTensors];
    int32_t block0[kSgdMaxTensors + 1];
    int32_t first[kSgdMaxTensors];
    int32_t count;
};

template <int DT>
__device__ __forceinline__ float add_alpha16(float a, float b, float al, bool tail) {
    const float prod = __fmul_rn(b, al);
    return round16<DT>(__fadd_rn(a, tail ? round16<DT>(prod) : prod));
}

template <int DT, bool WD, bool MOM>
__global__ void __launch_bounds__(kBlock) k_sgd16(Sgd16Table t, SgdHyper h) {
    int ti = 0;
    while (ti + 1 < t.count && (int)blockIdx.x >= t.block0[ti + 1]) ++ti;
    uint16_t* __restrict__ p = t.p[ti];
    const uint16_t* __restrict__ g = t.g[ti];
    uint16_t* __restrict__ buf = t.buf[ti];
    const int64_t n = t.n[ti];
    const int64_t body = n - n % 32;
    const bool first = t.first[ti] != 0;
    // alphas rounded to the dtype (the CPU kernels' scalar_t alpha)
    const float a_damp = round16<DT>(h.damp_alpha), a_mom = round16<DT>(h.mom), a_lr = round16<DT>(h.neg_lr);
    const int64_t base = (int64_t)(blockIdx.x - t.block0[ti]) * kSgd16PerBlock;
#pragma unroll
    for (int u = 0; u < kSgd16PerThread; ++u) {
        const int64_t i = base + (int64_t)u * kBlock + threadIdx.x;
        if (i >= n) break;
        const bool tail = i >= body;
        const float pv = h16_to_f32<DT>(p[i]), gv = h16_to_f32<DT>(g[i]);
        float d = gv;
        if (WD) {
            d = round16<DT>(__fmul_rn(pv, h.wd));                        // weight_decay * p.data
            if (MOM) {
                float b;
                if (first) {
                    b = d;                                               // buf = d_p
                } else {
                    b = round16<DT>(__fmul_rn(h16_to_f32<DT>(buf[i]), h.mom));   // buf.mul_(momentum)
                    b = add_alpha16<DT>(b, d, a_damp, tail);             // .add_(d_p, alpha=1 - dampening)
                }
                buf[i] = f32_to_h16<DT>(b);
                d = h.nesterov ? add_alpha16<DT>(d, b, a_mom, tail) : b;
            }
            d = round16<DT>(__fadd_rn(d, gv));                           // d_p.add(p.grad)
        }
        p[i] = f32_to_h16<DT>(add_alpha16<DT>(pv, d, a_lr, tail));       // p.add_(d_p, alpha=-lr)
    }
}

}  // namespace dgc

extern "C" int dgc_sgd_step16(void* const* params, const void* const* grads, void* const* bufs,
                              const int64_t* numels, const int32_t* first, int32_t count, float lr, float momentum,
                              float dampening, float weight_decay, int32_t nesterov, int32_t dtype, void* stream) {
    using namespace dgc;
    if (count < 0 || (count > 0 && (!params || !grads || !numels)))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step16: null tensor table");
    if (dtype != DGC_BF16 && dtype != DGC_F16) DGC_FAIL(DGC_ERR_DTYPE, "dgc_sgd_step16: dtype must be bf16 or fp16");
    const bool wd = weight_decay != 0.f, mom = wd && momentum != 0.f;
    if (mom && (!bufs || !first)) DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step16: momentum needs buffers");
    SgdHyper h{weight_decay, momentum, 1.f - dampening, -lr, nesterov};
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int32_t c0 = 0; c0 < count; c0 += kSgdMaxTensors) {
        Sgd16Table t{};
        int64_t blocks = 0;
        for (int32_t j = 0; j < kSgdMaxTensors && c0 + j < count; ++j) {
            const int32_t i = c0 + j;
            if (!params[i] || !grads[i] || numels[i] < 0 || (mom && !bufs[i]))
                DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step16: tensor %d: null pointer or n < 0", i);
            t.p[t.count] = static_cast<uint16_t*>(params[i]);
            t.g[t.count] = static_cast<const uint16_t*>(grads[i]);
            t.buf[t.count] = mom ? static_cast<uint16_t*>(bufs[i]) : nullptr;
            t.n[t.count] = numels[i];
            t.first[t.count] = mom ? first[i] : 0;
            t.block0[t.count] = (int32_t)blocks;
            blocks += ceil_div(numels[i], (int64_t)kSgd16PerBlock);
            if (blocks > 0x7FFFFFFF) DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step16: too many elements in one group");
            t.count++;
        }
        t.block0[t.count] = (int32_t)blocks;
        if (blocks == 0) continue;
        const dim3 gd((unsigned)blocks), bd(kBlock);
#define DGC_SGD16(D) \
        if (!wd) hipLaunchKernelGGL((k_sgd16<D, false, false>), gd, bd, 0, s, t, h); \
        else if (!mom) hipLaunchKernelGGL((k_sgd16<D, true, false>), gd, bd, 0, s, t, h); \
        else hipLaunchKernelGGL((k_sgd16<D, true, true>), gd, bd, 0, s, t, h);
        if (dtype == DGC_BF16) {
            DGC_SGD16(DGC_BF16)
        } else {
            DGC_SGD16(DGC_F16)
        }
#undef DGC_SGD16
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

extern "C" int dgc_sgd_step(float* const* params, const float* const* grads, float* const* bufs,
                            const int64_t* numels, const int32_t* first, int32_t count, float lr, float momentum,
                            float dampening, float weight_decay, int32_t nesterov, void* stream) {
    using namespace dgc;
    if (count < 0 || (count > 0 && (!params || !grads || !numels)))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step: null tensor table");
    const bool wd = weight_decay != 0.f, mom = wd && momentum != 0.f;
    if (mom && (!bufs || !first)) DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step: momentum needs buffers");
    SgdHyper h{weight_decay, momentum, 1.f - dampening, -lr, nesterov};
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int32_t c0 = 0; c0 < count; c0 += kSgdMaxTensors) {
        SgdTable t{};
        int64_t blocks = 0;
        for (int32_t j = 0; j < kSgdMaxTensors && c0 + j < count; ++j) {
            const int32_t i = c0 + j;
            if (!params[i] || !grads[i] || numels[i] < 0 || (mom && !bufs[i]))
                DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step: tensor %d: null pointer or n < 0", i);
            t.p[t.count] = params[i];
            t.g[t.count] = grads[i];
            t.buf[t.count] = mom ? bufs[i] : nullptr;
            t.n[t.count] = numels[i];
            t.first[t.count] = mom ? first[i] : 0;
            t.block0[t.count] = (int32_t)blocks;
            blocks += ceil_div(numels[i], (int64_t)kSgdPerBlock);
            if (blocks > 0x7FFFFFFF) DGC_FAIL(DGC_ERR_INVALID, "dgc_sgd_step: too many elements in one group");
            t.count++;
        }
        t.block0[t.count] = (int32_t)blocks;
        if (blocks == 0) continue;
        if (!wd)
            hipLaunchKernelGGL((k_sgd<false, false>), dim3((unsigned)blocks), dim3(kBlock), 0, s, t, h);
        else if (!mom)
            hipLaunchKernelGGL((k_sgd<true, false>), dim3((unsigned)blocks), dim3(kBlock), 0, s, t, h);
        else
            hipLaunchKernelGGL((k_sgd<true, true>), dim3((unsigned)blocks), dim3(kBlock), 0, s, t, h);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}
