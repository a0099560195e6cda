/*
 * dgc_hip.h — C ABI of libdgc_hip.so, the MI355X (gfx950) DGC hot path.
 *
 * Every entry point replaces a piece of the reference's PyTorch/Horovod path
 * (emma-mens/adam-compression, paths relative to the reference root):
 *
 *   dgc_compensate        DGCSGDMemory.compensate            dgc/memory.py:50-70
 *                         (+ the strided sample of _sparsify  dgc/compression.py:113,119)
 *   dgc_sample_strided    importance[start::stride]          dgc/compression.py:113,119
 *   dgc_sample_gather     importance[randint(...)]           dgc/compression.py:120-121
 *   dgc_kth_largest       min(topk(samples, k))              dgc/compression.py:123
 *   dgc_mask_indices      DGCSGDMemory.update                dgc/memory.py:72-77
 *   dgc_select            ge/nonzero + adaptation loop +     dgc/compression.py:124-153
 *                         resample + truncate + gather,
 *                         DGCSGDMemory.update,               dgc/memory.py:72-77
 *                         wire casts                         dgc/compression.py:168-171
 *   dgc_compress          compensate -> _sparsify -> update  dgc/compression.py:155-172
 *   dgc_decompress        zero_ + index_put_(accumulate)     dgc/compression.py:179-194
 *                         + mul_(1/W) over the rank-order
 *                         concatenation of the allgather     dgc/compression.py:200-212
 *   dgc_decompress_packed the same, straight from the padded RCCL allgather buffer
 *   dgc_scatter_packed    its sparse form (zero_() done earlier by dgc_fill_zero)
 *   dgc_decompress_packed_over  the same into a persistent output that holds the
 *                         previous call's result (zero_() as a sparse re-zero);
 *                         dgc_clear_packed + dgc_scatter_packed_cleared: its two halves
 *   dgc_sgd_step          DGCSGD.step (weight-decay momentum + update) dgc/optim/sgd.py:42-68
 *   dgc_compensate16, dgc_mask_indices16, dgc_widen16, dgc_decompress16
 *                         the same memory / decompress for bf16 / fp16 parameters
 *                         (dgc/memory.py:43-77, dgc/compression.py:179-194 on a
 *                         16-bit tensor: every op rounds to the dtype)
 *
 * Conventions
 *   - All tensor pointers are DEVICE pointers owned by the caller (PyTorch's caching
 *     allocator). The library never allocates; scratch comes from a caller-supplied
 *     workspace whose size the *_workspace() queries return. Workspaces must be
 *     256-byte aligned.
 *   - Every call is stream-ordered on `stream` (a hipStream_t; NULL = legacy stream)
 *     and returns immediately, except dgc_compress / dgc_select with
 *     DGC_SYNC_HOST, which read a few bytes of device state back to skip kernels.
 *   - Return value: DGC_OK or an error code; dgc_last_error() gives a thread-local
 *     message. Kernel faults surface at the caller's next synchronisation.
 *   - Element counts are int64: the 7B-element buckets exceed 2^32.
 */
#ifndef DGC_HIP_H
#define DGC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum dgc_status {
    DGC_OK = 0,
    DGC_ERR_INVALID = 1,      /* bad argument (null pointer, k > n, ...) */
    DGC_ERR_DTYPE = 2,        /* unsupported value / index dtype */
    DGC_ERR_OVERFLOW = 3,     /* int32 indices requested for n > 2^31 - 1, or a    */
                              /* resample replay that cannot address the tensor:   */
                              /* more than 2^32 - 1 candidates (min(64k - 1, n);   */
                              /* resample = 1 only)                                */
    DGC_ERR_HIP = 4,          /* a HIP runtime call failed */
    DGC_ERR_WORKSPACE = 5,    /* workspace too small or misaligned */
    DGC_ERR_UNSORTED = 6      /* decompress input has more descending runs than supported */
};

enum dgc_vdtype { DGC_F32 = 0, DGC_F16 = 1, DGC_BF16 = 2 };   /* value / parameter dtype; wire values:
                                                 fp16_values -> F16, else the param dtype */
enum dgc_idtype { DGC_I64 = 0, DGC_I32 = 1 };   /* wire index dtype  (int32_indices) */

enum dgc_sync_mode {
    DGC_SYNC_DEVICE = 0,      /* every decision on device; no host synchronisation      */
    DGC_SYNC_HOST = 1         /* read decisions back to skip unneeded launches (drop-in) */
};

/* Branch taken by the selection (mirrors the reference's adaptation loop). */
enum dgc_branch {
    DGC_BRANCH_DIRECT = 0,    /* numel == num_samples: no adaptation loop */
    DGC_BRANCH_OK = 1,        /* lower*k <= n <= k                        */
    DGC_BRANCH_TRUNC = 2,     /* k < n <= upper*k: first k ascending      */
    DGC_BRANCH_RESAMPLE = 3,  /* n > upper*k: top-k of the candidates     */
    DGC_BRANCH_EXHAUSTED = 4  /* max_adaptation_iters recounts used up    */
};

/* How a resample chose among the candidates tied at its k-th value: torch's CPU topk
 * replayed exactly, on both of its paths (nth_element for k*64 > n candidates,
 * partial_sort otherwise) — the reference's indices in the reference's order; or, for a
 * caller that asked for index order (resample_order = 1) when the k-th largest key is
 * not tied across the k boundary, the same SET in ascending index order. */
enum dgc_tie_rule {
    DGC_TIES_NONE = 0,   /* no resample this call */
    DGC_TIES_EXACT = 1,  /* torch's topk replayed */
    DGC_TIES_SET = 2     /* untied boundary: topk's set, index order */
};

/* Per-tensor selection parameters: DGCCompressor.attributes[name]
 * (dgc/compression.py:85) plus the compressor's knobs (dgc/compression.py:18-54). */
typedef struct dgc_select_params {
    int64_t numel;            /* N                                          */
    int64_t num_selects;      /* k = ceil(N * ratio)                        */
    int64_t num_samples;      /* attributes num_samples (N == S: no loop)   */
    int64_t upper_count;      /* floor(k * compress_upper_bound)  (n > U)   */
    int64_t lower_count;      /* ceil(compress_lower_bound * k)   (n < L)   */
    float upper;              /* fl32(compress_upper_bound), threshold *=   */
    float lower;              /* fl32(compress_lower_bound), threshold *=   */
    int32_t max_iters;        /* max_adaptation_iters                       */
    int32_t resample;         /* resample flag                              */
    int32_t masking;          /* DGCSGDMemory.momentum_masking               */
    int32_t vdtype;           /* enum dgc_vdtype of values_out              */
    int32_t idtype;           /* enum dgc_idtype of indices_out             */
    int32_t update_memory;    /* 1: zero the emitted slots of vec (and of   */
                              /*    mmt when masking) = DGCSGDMemory.update */
                              /* 2 (dgc_compress only): deferred — the next */
                              /*    dgc_compress_begin on this workspace    */
                              /*    zeroes them while it streams vec/mmt;   */
                              /*    dgc_compress_flush applies it on demand */
                              /* 0: pure selection, vec/mmt untouched       */
    int32_t thr_dtype;        /* dtype of the tensor being sparsified        */
                              /* (DGC_F32 / DGC_BF16 / DGC_F16): the        */
                              /* threshold *= bound products round to it,   */
                              /* as the 0-dim threshold tensor does          */
    int32_t resample_order;   /* 0: a resample lists torch.topk's order (the    */
                              /*    exact replay); 1: index order when the k-th */
                              /*    largest candidate key is untied (DGC_TIES_  */
                              /*    SET: the same set, for an engine whose      */
                              /*    decompress / update depend on the set only)  */
    int32_t* status_sink;     /* NULL, or a host-mapped (pinned) int32: a call  */
                              /* whose resample replay broke stores its       */
                              /* dgc_select_info.k5_status there (with        */
                              /* DGC_K5_BROKEN set) — nothing is written      */
                              /* otherwise — so a DGC_SYNC_DEVICE caller can  */
                              /* check every step without synchronising       */
    int64_t* order_out;       /* NULL, or a device int64 the call sets to        */
                              /* DGC_ORDER_ASCENDING when its emitted indices    */
                              /* ascend (no exact-replay topk order), else 0 —   */
                              /* an engine points it at its packed payload's     */
                              /* header word 1, which the W = 1 scatter reads    */
} dgc_select_params;

/* Packed payload header word 1 of an engine payload whose indices ascend: the W = 1
 * decompress then writes whole 64-B granules (dgc_batch_compress_finish and
 * dgc_batch_select set it on their payload; dgc_select / dgc_compress* through
 * dgc_select_params.order_out). */
#define DGC_ORDER_ASCENDING 0x444E454353413147LL

/* Device-resident result record written by dgc_select / dgc_compress. */
typedef struct dgc_select_info {
    int64_t count;            /* n emitted (== *count_out)                  */
    int64_t candidates;       /* count at the final threshold               */
    float threshold0;         /* sampled threshold                          */
    float threshold;          /* final threshold                            */
    int32_t branch;           /* enum dgc_branch                            */
    int32_t recounts;         /* adaptation recounts executed               */
    int32_t overflow_segments;/* segments whose candidate list spilled      */
    int32_t full_passes;      /* full re-reads of vec (0: served by the K1 lists) */
    int32_t tie_rule;         /* enum dgc_tie_rule                          */
    int32_t window_keys;      /* > 0: threshold0 came from the K1 window list of this
                                 many samples (those >= the list threshold), not a
                                 pass over all samples; same value either way       */
    int32_t k5_status;        /* resample replay: bit 0 (DGC_K5_FALLBACK) the multi-
                                 workgroup global phase found its workgroups not all
                                 resident and left the whole replay to one workgroup
                                 (exact, slower); bit 2 (DGC_K5_RECOVERED) a barrier of
                                 that phase timed out after it had started, so the call
                                 rebuilt the candidate queue and replayed it on one
                                 workgroup from scratch (exact, in the same call); bit 1
                                 (DGC_K5_BROKEN) a replay that could not be recovered:
                                 the selection of this tensor is NOT reliable (the
                                 engines raise) — not produced by this library version */
    float list_threshold;     /* the K1 candidate lists' threshold this call used (+inf:
                                 none); diagnostics of the speculative listing       */
} dgc_select_info;

/* bit 3 (DGC_K5_SET_FALLBACK): the batch engines' multi-workgroup set path (K5s)
   found its workgroups not all resident and left the tensor to the exact replay; bit 4
   (DGC_K5_SET_BROKEN): a K5s barrier timed out, the replay took the tensor (exact
   either way — counted by the engines' selection records) */
enum { DGC_K5_FALLBACK = 1, DGC_K5_BROKEN = 2, DGC_K5_RECOVERED = 4, DGC_K5_SET_FALLBACK = 8,
       DGC_K5_SET_BROKEN = 16 };

const char* dgc_last_error(void);
const char* dgc_version(void);

/* ---- K1: momentum correction + velocity accumulation (+ fused strided sample) ----
 * accumulate=1: mmt, vec updated in place, out must be NULL or == vec.
 * accumulate=0: mmt updated, result written to out (vec unused).
 * samples != NULL: samples[q] = |vec_new[sample_start + q*sample_stride]| for
 *                  q < num_samples (num_samples = ceil((n - start) / stride)). */
int dgc_compensate(const float* grad, float* mmt, float* vec, float* out, int64_t n,
                   float momentum, int32_t nesterov, int32_t accumulate,
                   float* samples, int64_t sample_start, int64_t sample_stride,
                   int64_t num_samples, void* stream);

/* DGCSGDMemory.update (dgc/memory.py:72-77) as a standalone scatter: vec[i] = 0 and,
 * when mmt != NULL (momentum_masking), mmt[i] = 0 for i in indices[0..count).
 * Negative indices wrap like torch (index_fill_); an index outside [-n, n) — where the
 * reference's index_fill_ raises (dgc/memory.py:76-77) — is skipped and sets *bad_flag:
 * a device int32 or a host-mapped (pinned) one the caller polls without synchronising;
 * the library stores 1 there (never clears it). */
int dgc_mask_indices(float* mmt, float* vec, int64_t n, const void* indices, int32_t idtype,
                     int64_t count, int32_t* bad_flag, void* stream);

/* ---- K2: sampling ---- */
int dgc_sample_strided(const float* vec, int64_t n, int64_t start, int64_t stride,
                       float* samples, int64_t num_samples, void* stream);
int dgc_sample_gather(const float* vec, const int64_t* sample_indices, int64_t num_samples,
                      float* samples, void* stream);

/* ---- K3: k-th largest of |x| (topk threshold); NaN if any |x| is NaN ---- */
size_t dgc_kth_largest_workspace(int64_t n);
int dgc_kth_largest(const float* x, int64_t n, int64_t k, float* thr_out,
                    void* ws, size_t ws_bytes, void* stream);

/* ---- K4: selection, adaptation loop, pack, masking ----
 * vec (length numel) is read; with params.update_memory its emitted slots are
 * zeroed, and mmt's too when params.masking (dgc_compress forces update_memory=1). thr0 is the device scalar from dgc_kth_largest. Writes
 * values_out[0..n), indices_out[0..n) (ascending), *count_out = n (device int64)
 * and *info_out (device, may be NULL). */
size_t dgc_select_workspace(int64_t numel, int64_t num_selects);
int dgc_select(float* vec, float* mmt, const float* thr0, const dgc_select_params* params,
               void* values_out, void* indices_out, int64_t* count_out,
               dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
               void* stream);

/* ---- fused compress: compensate + sample + threshold + select ----
 * Speculative listing: K1 also lists every element with |vec_new| >= spec_threshold[0]
 * into the selection workspace. spec_threshold is a device float[8], in/out, per
 * tensor (NULL = off); initialise all eight to +inf. When the sampled threshold comes out
 * >= spec[0] and few segment lists overflowed, every count and selection is served
 * from the lists and the separate re-read of vec is skipped; otherwise one full pass
 * runs. Results are identical either way (spec only chooses the work).
 * On return spec[1] = the final threshold t and spec[0] = m x t x growth, growth =
 * 2 - (previous t) / t (linear extrapolation) clamped to [1, 1.5]; m = spec_margin (0.8
 * is a good one) after a call whose t fell below its list threshold, else 1.05 x (list
 * threshold / t) of that call, within [spec_margin, spec[4]]: the lists shrink while t
 * moves predictably. spec[4], the ceiling, starts at 0.95 and moves within
 * [spec_margin, 0.985]: +0.005 after every call whose t held at or above its list
 * threshold, -0.05 after one that fell below it. spec[2..3] predict the sampled
 * threshold for K1's sample window (spec[2] = the window threshold, spec[3] = the last
 * sampled threshold); spec[5..7] are reserved.
 * dgc_compress = dgc_compress_begin (K1) + dgc_compress_finish (K3, K4), which share
 * one workspace and must see the same sample_start/stride/params. The workspace
 * carries per-tensor state from call to call (a deferred masking, the K1 list-spill
 * and sample-window counts): zero-fill it before its first call, and give each
 * tensor its own. */
size_t dgc_compress_workspace(int64_t numel, int64_t num_selects, int64_t num_samples);
int dgc_compress(const float* grad, float* mmt, float* vec, float momentum, int32_t nesterov,
                 int64_t sample_start, int64_t sample_stride, int64_t top_k_samples,
                 const dgc_select_params* params, float* spec_threshold, float spec_margin,
                 void* values_out, void* indices_out, int64_t* count_out, dgc_select_info* info_out,
                 void* ws, size_t ws_bytes, int32_t sync_mode, void* stream);
int dgc_compress_begin(const float* grad, float* mmt, float* vec, float momentum, int32_t nesterov,
                       int64_t sample_start, int64_t sample_stride, const dgc_select_params* params,
                       const float* spec_threshold, void* ws, size_t ws_bytes, void* stream);
int dgc_compress_finish(float* vec, float* mmt, int64_t sample_start, int64_t sample_stride,
                        int64_t top_k_samples, const dgc_select_params* params, float* spec_threshold,
                        float spec_margin, void* values_out, void* indices_out, int64_t* count_out,
                        dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                        void* stream);
/* Applies a masking that a dgc_compress_finish with params.update_memory == 2 left
 * pending on this workspace (no-op when none is). Call before reading vec/mmt (state
 * dict, checkpoint) between a dgc_compress_finish and the next dgc_compress_begin
 * (which applies it by itself; a flush after that begin would zero the new values). */
int dgc_compress_flush(float* vec, float* mmt, int64_t sample_stride, const dgc_select_params* params,
                       void* ws, size_t ws_bytes, void* stream);

/* ---- batch: every compressed tensor of a step in the same launches ----
 * The reference compresses tensor by tensor from the optimizer's hooks
 * (dgc/horovod/optimizer.py:116-155). A batch lays its `count` tensors at offsets of
 * three flat fp32 buffers (grad, mmt, vec; offsets multiples of 1024, ascending,
 * each tensor followed by zeros up to a multiple of 4) and runs compensate ->
 * sample -> threshold -> select / adapt / resample -> pack -> masking for all of
 * them with O(1) launches per phase and, in DGC_SYNC_DEVICE mode, no host sync.
 * Per tensor the numerics are exactly dgc_compress's (same attributes, same
 * sample start). The payload is ONE packed rank buffer (dgc_payload_layout with
 * capacity = sum of num_selects): the tensors' entries one after the other, in
 * tensor order, with FLAT indices (offset + index in the tensor); decompress it with
 * dgc_decompress_packed / dgc_scatter_packed over flat_numel elements. */
typedef struct dgc_batch_desc {
    int32_t count;                  /* tensors                                        */
    const int64_t* numel;           /* host arrays of `count`: attributes per tensor  */
    const int64_t* offset;          /*   (dgc/compression.py:85)                      */
    const int64_t* num_selects;
    const int64_t* num_samples;
    const int64_t* top_k_samples;
    const int64_t* sample_stride;
    int64_t flat_numel;             /* length of the flat buffers                     */
    double upper_bound, lower_bound;/* compress_upper_bound / compress_lower_bound    */
    int32_t max_iters, resample, momentum_masking, fp16_values, int32_indices, nesterov;
    float momentum;
    float spec_margin;              /* speculative list threshold margin (0.8)        */
    int32_t deferred_masking;       /* 1: first-k branches leave DGCSGDMemory.update's */
                                    /*   zeroing to the next compress's K1 (which    */
                                    /*   streams vec/mmt anyway); dgc_batch_flush    */
                                    /*   applies it before vec/mmt are read elsewhere */
    int32_t dtype;                  /* parameter dtype: DGC_F32 (0: dgc_batch_compress*), */
                                    /*   DGC_BF16 / DGC_F16 (dgc_batch_select over the  */
                                    /*   dgc_compensate16 image, 16-bit wire values     */
                                    /*   unless fp16_values, dgc_mask_packed16,         */
                                    /*   dgc_decompress_packed16)                       */
    int32_t resample_order;         /* as dgc_select_params.resample_order             */
    int32_t* status_sink;           /* as dgc_select_params.status_sink (NULL: none)   */
} dgc_batch_desc;

size_t dgc_batch_workspace(const dgc_batch_desc* batch);
/* Writes the batch's device tables into the workspace (synchronous). Re-run after any
 * change of the tensors or their attributes (e.g. warmup_compress_ratio). */
int dgc_batch_init(const dgc_batch_desc* batch, void* ws, size_t ws_bytes, void* stream);
/* sample_starts: host array of `count` (random.randint(0, stride - 1) per tensor, in
 * the tensors' order); info_out: device array of `count` records (may be NULL). */
int dgc_batch_compress(const dgc_batch_desc* batch, const float* grad, float* mmt, float* vec,
                       const int64_t* sample_starts, void* payload, dgc_select_info* info_out, void* ws,
                       size_t ws_bytes, int32_t sync_mode, void* stream);
/* dgc_batch_compress in its two phases (same arguments): begin = K1 over every tensor
 * (compensate + strided samples + speculative candidate lists, and any masking a
 * deferring finish left pending); finish = K3 thresholds + the selection into the
 * payload. Nothing may touch grad/mmt/vec between them. */
int dgc_batch_compress_begin(const dgc_batch_desc* batch, const float* grad, float* mmt, float* vec,
                             const int64_t* sample_starts, void* ws, size_t ws_bytes, void* stream);
/* dgc_batch_compress_begin with the gradients taken where they are: grads is a HOST
 * array of `count` device pointers, grads[t] holding numel[t] contiguous floats, 16-B
 * aligned (the parameters' own p.grad tensors as autograd left them — the batched
 * DistributedOptimizer, dgc/horovod/optimizer.py:116-155, without a copy into the flat
 * buffer). A tensor that ends inside a float4 is read to its last element only. */
int dgc_batch_compress_begin_ptrs(const dgc_batch_desc* batch, const float* const* grads, float* mmt, float* vec,
                                  const int64_t* sample_starts, void* ws, size_t ws_bytes, void* stream);
int dgc_batch_compress_finish(const dgc_batch_desc* batch, float* mmt, float* vec, void* payload,
                              dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                              void* stream);
/* The selection of a batch over a flat fp32 buffer that no dgc_batch_compress_begin
 * produced — a 16-bit batch's velocity image from dgc_compensate16 (vec32 = its
 * vec32 output over the flat 16-bit buffers): the strided samples, the thresholds and
 * the selection into the payload, as dgc_batch_compress_finish (no candidate lists).
 * A 16-bit batch (desc dtype) leaves vec32 untouched (mmt32 may be NULL); mask its
 * state with dgc_mask_packed16. */
int dgc_batch_select(const dgc_batch_desc* batch, float* vec32, float* mmt32, const int64_t* sample_starts,
                     void* payload, dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                     void* stream);
/* Pending deferred masking (deferred_masking = 1) applied now; no-op when none is. */
int dgc_batch_flush(const dgc_batch_desc* batch, float* mmt, float* vec, void* ws, size_t ws_bytes, void* stream);

/* ---- K6: deterministic decompress ----
 * grad[0..n) = scale * (rank-order sequential sum of the entries), every other
 * slot +0.0. dgc_decompress takes the concatenated (values, indices) of the
 * allgather; run_offsets (HOST array of nruns+1 entry offsets, e.g. the per-rank
 * counts' prefix sums) may be NULL, in which case runs are detected on device. */
size_t dgc_decompress_workspace(int64_t n, int32_t max_runs);
int dgc_decompress(const void* values, int32_t vdtype, const void* indices, int32_t idtype,
                   int64_t total, const int64_t* run_offsets, int32_t nruns,
                   float* grad, int64_t n, float scale, void* ws, size_t ws_bytes, void* stream);

/* Packed per-rank payload (the RCCL allgather unit), byte offsets from the
 * rank's base:  [0] int64 count | [values_offset] values | [indices_offset] indices;
 * rank r starts at payload + r * rank_stride. */
int64_t dgc_payload_layout(int64_t capacity, int32_t vdtype, int32_t idtype,
                           int64_t* values_offset, int64_t* indices_offset);
/* Workspace of dgc_decompress_packed / dgc_scatter_packed: it includes the area in
 * which a rank's run that is not in ascending index order (the reference's resample
 * sends torch.topk's order, dgc/compression.py:134-137) is regrouped by chunk. */
size_t dgc_decompress_packed_workspace(int64_t n, int32_t world, int64_t capacity);
int dgc_decompress_packed(const void* payload, int32_t world, int64_t rank_stride,
                          int64_t capacity, int32_t vdtype, int32_t idtype,
                          float* grad, int64_t n, float scale, void* ws, size_t ws_bytes,
                          void* stream);
/* Sparse form of dgc_decompress_packed: grad must already hold +0.0 everywhere (the
 * reference's grad.zero_(), dgc/compression.py:191, issued earlier — e.g. with
 * dgc_fill_zero on a second stream while compress and the allgather run); only the
 * indices present are written, with the same run-order sums and scale. */
int dgc_scatter_packed(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity,
                       int32_t vdtype, int32_t idtype, float* grad, int64_t n, float scale, void* ws,
                       size_t ws_bytes, void* stream);
/* dgc_decompress_packed into a PERSISTENT output: grad must hold exactly the result
 * of the previous decompress over `prev_payload` (same world / rank_stride / capacity /
 * dtypes / n, a different buffer than `payload`) and nothing else since, so it is +0.0
 * everywhere but at prev's indices. Those W*k slots are re-zeroed (the reference's
 * zero_(), dgc/compression.py:191, for W*k/n of the dense fill's traffic), then the
 * entries of `payload` are written as dgc_decompress_packed writes them: the dense
 * result is identical. The caller owns the precondition (dgc.bucket.DGCBucket checks
 * the output tensor's identity and version counter and falls back to the dense fill). */
int dgc_decompress_packed_over(const void* payload, const void* prev_payload, int32_t world,
                               int64_t rank_stride, int64_t capacity, int32_t vdtype, int32_t idtype,
                               float* grad, int64_t n, float scale, void* ws, size_t ws_bytes,
                               void* stream);
/* dgc_decompress_packed_over in two calls, so the re-zero can run on another stream
 * while the compress and the allgather run: dgc_clear_packed re-zeroes prev_payload's
 * entries in grad (same precondition) and resets the status words of `ws` (the
 * dgc_decompress_packed_workspace of the scatter to come); dgc_scatter_packed_cleared
 * then writes the new payload's entries, ordered after the clear by the caller, with
 * that workspace untouched in between. */
int dgc_clear_packed(const void* prev_payload, int32_t world, int64_t rank_stride, int64_t capacity,
                     int32_t vdtype, int32_t idtype, float* grad, int64_t n, void* ws, size_t ws_bytes,
                     void* stream);
int dgc_scatter_packed_cleared(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity,
                               int32_t vdtype, int32_t idtype, float* grad, int64_t n, float scale, void* ws,
                               size_t ws_bytes, void* stream);
/* grad[0..n) = +0.0 with one-shot 16-B stores (4-B aligned buffer; a scalar head up to
 * the first 16-B boundary). */
int dgc_fill_zero(float* grad, int64_t n, void* stream);

/* ---- split exchange: the allgather of dgc/compression.py:200-212 in `parts` collectives
 * (2..8), the decompress of what has landed running while the rest is in flight ----
 * dgc_payload_split re-lays a rank's packed payload (capacity entries) out as `parts`
 * part buffers of dgc_payload_split_layout bytes each, consecutive: part p is a packed
 * payload (dgc_payload_layout(part_capacity)) of the entries [p * part_capacity,
 * (p + 1) * part_capacity) whose header holds [0] its count and [1] the smallest index
 * in the parts after it (INT64_MAX: none). `split` is dgc_payload_split_bytes long
 * (the parts, then scratch that must be zero before the first call; calls leave it zero).
 * Part p is allgathered into gathered + p * world * part_bytes (rank r's at + r *
 * part_bytes: part-major). dgc_scatter_split(part p), called for p = 0, 1, ... in order
 * on one workspace after part p landed, writes every index below min over ranks of part
 * p's bound (and not below part p-1's) — such an index has all its entries in parts <= p
 * — with dgc_scatter_packed's sums: each index's run-order (rank-order) sum * scale, the
 * last call writing the rest. grad holds +0.0 before part 0: zero-filled (cleared = 0),
 * or re-zeroed by dgc_clear_split on this workspace (cleared = 1; same precondition as
 * dgc_clear_packed, over the previous step's split gathered buffer). */
int64_t dgc_payload_split_layout(int64_t capacity, int32_t parts, int32_t vdtype, int32_t idtype,
                                 int64_t* part_capacity);
int64_t dgc_payload_split_bytes(int64_t capacity, int32_t parts, int32_t vdtype, int32_t idtype);
int dgc_payload_split(const void* payload, int64_t capacity, int32_t parts, int32_t vdtype, int32_t idtype,
                      void* split, void* stream);
size_t dgc_decompress_split_workspace(int64_t n, int32_t world, int32_t parts, int64_t capacity);
int dgc_scatter_split(const void* gathered, int32_t world, int32_t parts, int32_t part, int64_t capacity,
                      int32_t vdtype, int32_t idtype, float* grad, int64_t n, float scale, int32_t cleared, void* ws,
                      size_t ws_bytes, void* stream);
int dgc_clear_split(const void* prev_gathered, int32_t world, int32_t parts, int64_t capacity, int32_t vdtype,
                    int32_t idtype, float* grad, int64_t n, void* ws, size_t ws_bytes, void* stream);

/* Status word written by the decompress kernels: bit 0 = an index was out of
 * range [0, n) and was ignored (the reference's index_put_ raises,
 * dgc/compression.py:191); bit 1 = a run was not non-decreasing; bit 2 = a packed
 * header's count was outside [0, capacity] (the run was clamped to it). Packed runs
 * are then regrouped and summed exactly (indices unique within a run); a run given by
 * run_offsets to dgc_decompress is not regrouped (its stray entries were ignored).
 * Reads 4 bytes from the workspace (synchronous). */
int dgc_decompress_status(const void* ws, int32_t* status, void* stream);
/* Binds a decompress workspace to two host-mapped (pinned) int32 words [index, count]:
 * every later decompress / scatter call on `ws` (dgc_decompress, dgc_decompress_packed,
 * _over, dgc_scatter_packed, _cleared, dgc_scatter_split) that meets status bit 0 also
 * stores 1 into sink[0], bit 2 into sink[1], from the kernel that finds it — so a
 * DGC_SYNC_DEVICE caller (the engines) raises at its next step, as the reference raises
 * at its index_put_, with no host synchronisation (nothing is written while the data are
 * healthy). The library never clears the words. sink = NULL unbinds; rebinding `ws`
 * replaces its binding. The binding is keyed by the workspace address: unbind before
 * the workspace is freed. */
int dgc_decompress_bind_sink(const void* ws, int32_t* sink);

/* Measurement only (bench.py): K1's memory shape — d = a + c, e = b + c over n
 * floats (n/4 float4; 16-B aligned buffers), three non-temporal 16-B reads and two
 * non-temporal 16-B writes per float4 — to measure the streaming rate of the box at
 * hand next to K1. Not part of the reference's interface. */
int dgc_hbm_probe(const float* a, const float* b, const float* c, float* d, float* e, int64_t n, void* stream);

/* ---- the dense (uncompressed) tensors of a step (dgc/compression.py:173-177, 195-198) ----
 * dgc_gather_cast: dst[offsets[t] + i] = (dst_dtype) srcs[t][i] for count tensors (HOST
 *   arrays; srcs[t]: numels[t] device floats, any alignment) — the dense gradients into
 *   one allreduce buffer, with compress's `tensor.type(torch.float16)` when dst_dtype is
 *   DGC_F16 (DGC_BF16 and DGC_F32 too), in one launch per 64 tensors.
 * dgc_compensate_wire: out = DGCSGDMemory.compensate(g, accumulate=False) (mmt updated),
 *   g = the exchanged gradient: src_dtype DGC_F16 (widened exactly, decompress's
 *   `tensor.type(vdtype)`) or DGC_F32; round_to = DGC_F16 with an fp32 src rounds it to
 *   fp16 and back first (a one-rank exchange of an fp16 wire without the buffer).
 * dgc_compensate_multi: the same from each tensor's own gradient (srcs[t], numels[t];
 *   HOST arrays) into mmt / out at offsets[t] of two flat buffers, round_to as above:
 *   a one-rank step's dense tensors in one launch per 64 tensors. */
int dgc_gather_cast(const float* const* srcs, const int64_t* numels, const int64_t* offsets, int32_t count,
                    void* dst, int32_t dst_dtype, void* stream);
int dgc_compensate_wire(const void* src, int32_t src_dtype, int32_t round_to, float* mmt, float* out, int64_t n,
                        float momentum, int32_t nesterov, void* stream);
/* dgc_compensate_wire_avg: the same from the allreduce's SUM over `world` ranks, the
 *   Average's division folded in (replaces horovod Average's post-division,
 *   dgc/compression.py:200-212 via hvd.allreduce_async_(op=Average)): g = src / world in
 *   fp32, rounded to fp16 for an fp16 src, as torch's `div_(world)` on the wire tensor. */
int dgc_compensate_wire_avg(const void* src, int32_t src_dtype, int32_t world, float* mmt, float* out, int64_t n,
                            float momentum, int32_t nesterov, void* stream);
int dgc_compensate_multi(const float* const* srcs, const int64_t* numels, const int64_t* offsets, int32_t count,
                         int32_t round_to, float* mmt, float* out, float momentum, int32_t nesterov, void* stream);
/* The dense Average of an ALLGATHER, summed in rank order (replaces Horovod's
 * allreduce_async_(op=Average), dgc/compression.py:205-206; the oracle's restatement:
 * acc = x_0; acc += x_1 ... x_{W-1}; acc /= W, each op on a tensor of the wire dtype —
 * an allreduce sums in the backend's order, which decides the last bits at W >= 3).
 * Rank r's n wire values (dtype DGC_F32 / DGC_F16 / DGC_BF16) start at src + r *
 * rank_stride BYTES. Every add rounds to the wire dtype; the division is the fp32 true
 * quotient by world (torch's CPU div_), rounded to the wire dtype.
 * dgc_rank_sum: dst[0..n) = that sum (/ world when average != 0), in the wire dtype; dst
 *   may be one of the source rows (dgc.comm.allreduce_async_ writes the rank's own tensor).
 * dgc_compensate_ranks: out = DGCSGDMemory.compensate(Average, accumulate=False), mmt
 *   updated (dgc/compression.py:195-198 after the exchange; src_dtype DGC_F32 or DGC_F16,
 *   widened exactly) — the batched step's dense tensors, carried in the packed payload. */
int dgc_rank_sum(const void* src, int32_t dtype, int32_t world, int64_t rank_stride, int64_t n, int32_t average,
                 void* dst, void* stream);
int dgc_compensate_ranks(const void* src, int32_t src_dtype, int32_t world, int64_t rank_stride, float* mmt,
                         float* out, int64_t n, float momentum, int32_t nesterov, void* stream);

/* ---- K7: DGCSGD.step over `count` parameters of one group (dgc/optim/sgd.py:42-68) ----
 * params[i], grads[i] (and bufs[i], the momentum_buffer, when weight_decay != 0 and
 * momentum != 0) are fp32 device arrays of numels[i] elements; first[i] = 1 when the
 * buffer is created on this step (buf = wd * p). Rounding follows the reference's
 * torch-CPU ops (add with alpha is one fused multiply-add). Stream-ordered. */
int dgc_sgd_step(float* const* params, const float* const* grads, float* const* bufs, const int64_t* numels,
                 const int32_t* first, int32_t count, float lr, float momentum, float dampening,
                 float weight_decay, int32_t nesterov, void* stream);
/* K7-16: the same for bf16 / fp16 parameters (dtype DGC_BF16 / DGC_F16; params, grads,
 * bufs 16-bit arrays of that dtype): every op rounds to the dtype as the reference's
 * torch-CPU ops on a 16-bit tensor do — alpha rounded to the dtype; `add(alpha)` rounds
 * fl32(x + y * alpha) once in the first n - n % 32 elements of a tensor (the CPU
 * kernels' vector body) and rounds the product first in the last n % 32 (their scalar
 * tail) — the split of a ONE-thread AVX2 CPU run, which tests/golden/sgd16.* pins; the
 * per-chunk tails of a multi-threaded run, AVX512's 64-element body and a CUDA run's
 * single rounding are not reproduced (parity with those unpinned). */
int dgc_sgd_step16(void* const* params, const void* const* grads, void* const* bufs, const int64_t* numels,
                   const int32_t* first, int32_t count, float lr, float momentum, float dampening,
                   float weight_decay, int32_t nesterov, int32_t dtype, void* stream);

/* ---- 16-bit parameters (bf16 / fp16, dtype = DGC_BF16 / DGC_F16) ----
 * The reference's memory and compressor on a bf16 / fp16 parameter
 * (dgc/memory.py:43-77, dgc/compression.py:109-198): each ATen op computes in fp32 and
 * rounds to the dtype. Arrays are 16-bit device arrays of that dtype.
 * dgc_compensate16: DGCSGDMemory.compensate (dgc/memory.py:50-70), rounding after
 *   each op; with accumulate, vec32 (may be NULL) receives the new velocity's exact
 *   fp32 image, which dgc_sample_strided / dgc_kth_largest / dgc_select then take as
 *   the tensor (thr_dtype = dtype, vdtype = DGC_F16 for fp16_values else dtype).
 * dgc_mask_indices16: DGCSGDMemory.update (dgc/memory.py:72-77).
 * dgc_widen16: y = fp32 image of x (a 16-bit tensor handed to the selection).
 * dgc_decompress16: grad.zero_().index_put_([idx], values.type(dtype),
 *   accumulate=True).mul_(scale) (dgc/compression.py:179-194): runs (ranks) in order,
 *   each add rounded to the dtype; indices distinct within a run (as DGC payloads
 *   are); the mul_ is skipped for scale == 1. run_offsets: host array, nruns + 1.
 *   nruns = -1: ONE run, indices stably sorted (duplicates in their input order),
 *   run_offsets = {begin, end}: each index's entries are folded in order — input
 *   that does not come as distinct-index runs (index_put_'s serial order). */
int dgc_compensate16(const void* grad, void* mmt, void* vec, void* out, float* vec32, int64_t n, float momentum,
                     int32_t nesterov, int32_t accumulate, int32_t dtype, void* stream);
int dgc_mask_indices16(void* mmt, void* vec, int64_t n, const void* indices, int32_t idtype, int64_t count,
                       int32_t* bad_flag, void* stream);
int dgc_widen16(const void* x, float* y, int64_t n, int32_t dtype, void* stream);
int dgc_decompress16(const void* values, int32_t vdtype, const void* indices, int32_t idtype,
                     const int64_t* run_offsets, int32_t nruns, void* grad, int32_t dtype, int64_t n, float scale,
                     int32_t* bad_flag, void* stream);
/* The 16-bit batch (dgc_batch_desc.dtype): DGCSGDMemory.update of the entries of one
 * packed payload (its device count) on the flat 16-bit state — mmt may be NULL
 * (momentum_masking off); the decompress of W packed payloads into a flat 16-bit
 * gradient (zero fill, the runs in rank order with every add rounded, then the 1/W
 * scale rounded, as dgc_decompress16); and the 2-byte multi-tensor gather of 16-bit
 * gradients into the flat buffer (srcs / numels / offsets: HOST arrays). */
int dgc_mask_packed16(const void* payload, int64_t capacity, int32_t vdtype, int32_t idtype, void* mmt, void* vec,
                      int64_t n, void* stream);
int dgc_decompress_packed16(const void* payload, int32_t world, int64_t rank_stride, int64_t capacity,
                            int32_t vdtype, int32_t idtype, void* grad, int32_t dtype, int64_t n, float scale,
                            int32_t* bad_flag, void* stream);
/* bad_flag of dgc_mask_indices16 / dgc_decompress16 / dgc_decompress_packed16: a device
 * or host-mapped int32 that receives 1 when an index is outside [-n, n) (negative ones
 * wrap as in index_put_ / index_fill_; the packed form takes none below 0) and 2 when a
 * packed header's count is outside [0, capacity] (that run is skipped); never cleared. */
int dgc_gather16(const void* const* srcs, const int64_t* numels, const int64_t* offsets, int32_t count, void* dst,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DGC_HIP_H */
