// K4: selection — the `importance >= threshold` mask, `nonzero()`, the adaptation
// loop, resample, truncation, value gather, momentum masking and wire packing —
// plus the listing K1 of the fused compress and the K3 thresholds, for ONE tensor or
// for a BATCH of T tensors in the same launches.
//
// Reference: DGCCompressor._sparsify (dgc/compression.py:109-153),
// DGCSGDMemory.update (dgc/memory.py:72-77), compress's casts (dgc/compression.py:168-171),
// compress's call order (dgc/compression.py:155-172); the batch serves every
// compressed tensor of a step, which the reference handles one hook at a time
// (dgc/horovod/optimizer.py:116-155).
//
// Layout. A tensor's elements are cut into SEGMENTS of 1024; 1024 segments form a
// GROUP (the scan granule and one emit workgroup). In a batch the tensors sit at
// segment-aligned offsets of flat grad/mmt/vec buffers; segments and groups are
// numbered globally, and every launch maps each workgroup to ONE tensor through a
// prefix table of per-tensor block counts (task_of_block), so per-tensor state,
// per-tensor tickets and group atomics never mix tensors. Every segment owns a
// candidate list of kCap = 64 slots (u16 offset + fp32 value, ascending) and two
// exact counts: seg_lcnt at the LIST threshold t_list (complete iff <= kCap; a
// spilled segment is re-read from vec when needed) and seg_cnt at the current
// threshold t_cur >= t_list.
//
// Speculative listing. K1 lists candidates at t_list = margin x (the previous call's
// final threshold), per tensor. When the sampled threshold comes out >= t_list — the
// steady state — every count and selection is served from the lists and the separate
// 4 B/elem re-read of vec disappears; otherwise a full select pass at t_cur re-lists.
// Results are identical either way: a list at t_list holds EVERY element >= t_list.
//
//   count pass   t_cur >= t_list: one thread per segment counts its list entries
//                (spilled segments: one wave re-reads 1024 elements); else the full
//                select pass (16 non-temporal float4 loads in flight per lane).
//   decide       (1 workgroup per tensor): the reference's loop step (ok / trunc /
//                resample / lower / raise / exhausted) + scan of the group totals.
//                resample=True: the first "lower" hands over to ONE multi-threshold
//                pass; resample=False: a recount per step.
//   resample     torch's CPU topk replayed exactly: nth_element path (candidates <
//                64 k): the candidates are gathered in index order and the introselect
//                replayed (K5, introselect.hpp); partial_sort path: heap select +
//                sort_heap over vec (K5b, heap_select_wg).
//   emit         (1 workgroup per group): positions (after the tensors before it in
//                the batch), fp32/fp16 values, int64/int32 indices, masking writes.
//
// Everything is stream-ordered; in DGC_SYNC_DEVICE mode kernels that turn out to
// be unneeded early-exit on a device flag, so no host synchronisation happens.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

#include "radix_select.hpp"
#include "introselect.hpp"

namespace dgc {

constexpr int kSeg = 1024;                      // elements per segment
constexpr int kCap = 64;                        // list slots per segment (6.25 %)
// The lists of kLstTile consecutive segments interleave: entry e of segment s sits at
// lcol(s) + e * kLstTile, so a 128-B line holds entries 0..7 of four lists. The
// selection reads a list per segment (~7 entries at 1e-3): contiguous 256-B list slots
// cost a line per segment there, the interleave a line per four. The four segments of
// a tile are K1's (and the select pass's) four waves of one workgroup, so the tile's
// lines fill in one L2.
constexpr int kLstTile = 4;
__host__ __device__ __forceinline__ int64_t lcol(int64_t seg) {
    return (seg / kLstTile) * (kLstTile * kCap) + seg % kLstTile;
}
// Slot of entry e of segment seg (every list access goes through it; ntile = tiles of
// kLstTile segments in the workspace, for layouts that band the entries — one that put
// entries 0..7 of every tile in one dense array was measured and dropped: flat-1B 3.61 /
// 3.67 ms against 3.73 / 3.71 ms banded, ResNet-50 unchanged).
__host__ __device__ __forceinline__ int64_t lslot(int64_t seg, int64_t e, int64_t ntile) {
    (void)ntile;
    return lcol(seg) + e * kLstTile;
}
constexpr int kSegTiles = kSeg / (kWave * 4);   // 4 float4 per lane per segment
constexpr int kSuper = 4;                       // segments per wave in the full select pass
constexpr int kGroupSegs = 1024;                // segments per group (1M elements)
constexpr int kCountSegs = 4;                   // k_count_lists: segments per thread (a group per block)
constexpr int kSegPerBlock4 = kBlock / kWave;   // 4 waves per workgroup
constexpr int kSegPerBlock16 = kSegPerBlock4 * kSuper;
constexpr int kMaxLower = 16;                   // thresholds per multi-threshold pass
constexpr int kSpillShards = 64;
constexpr int kSpillDiv = 32;                   // lists dropped when > nseg/32 segments spill
constexpr int kQueuePerBlock = kBlock;          // K5 emit: outputs per workgroup
constexpr int kCapBlocks = 2048;                // grid-stride launches: blocks per whole bucket (one tensor)
constexpr int kCapBlocksBatch = 16384;          // ... per whole batch of several tensors
// The adaptive list margin's ceiling (k_sel_finish, spec[4]): kSpecCeil0 at first, up by
// kSpecCeilUp after every hit to kSpecMarginMax, down by kSpecCeilDown after a miss.
constexpr float kSpecCeil0 = 0.95f;
constexpr float kSpecMarginMax = 0.985f;
constexpr float kSpecCeilUp = 0.005f, kSpecCeilDown = 0.05f;
// K5s, the set path of an untied resample (resample_order = 1; see k_resample_set): one
// launch, workgroups per tensor by its candidate capacity (BT_SET) — one up to
// kSetCoopMin, kSetG up to kSetG x kSetCoopMin, up to kSetGBig beyond (VGG-16-BN's fc6) —
// kSetRegC rounds of 1024 keys per workgroup in registers (32 spilled the radix
// passes' registers to scratch), up to kSetRoundsMax rounds from L2 beyond.
constexpr int kSetG = 16;                       // the most workgroups of a set's minimum (DGC_SET_G)
constexpr int kSetGDefault = 4;                 // ... and the default: a cooperative set's fewest workgroups
constexpr int kSetGBig = 128;
constexpr int kSetRegC = 16;
constexpr int kSetRoundsMax = 64;
constexpr int64_t kSetCoopMin = (int64_t)kSetRegC * 1024;   // (kScanThreads keys per round)
// its radix select: two passes over key - key(t_cur), bits [kSetLo0, kSetSpan) clamped
// (the top bin takes every key past the span) then [0, kSetLo0)
constexpr int kSetSpan = 25, kSetLo0 = 13;
constexpr int kSetBins0 = 1 << (kSetSpan - kSetLo0), kSetBins1 = 1 << kSetLo0;   // 4096, 8192
constexpr int kSpecWords = 8;                   // per-tensor speculation state (dgc_compress_begin: spec)
constexpr int kChainOneWords = 256;             // SelWS::chain: k_chain_one's words (zeroed every call) ...
constexpr int kChainWords = kChainOneWords + 128;   // ... then k_rs_passes' (zero at rest)
constexpr int kEmitSplit = 4;                   // k_emit workgroups per group
constexpr int64_t kSetOneMax = kSetCoopMin;     // K5s: one workgroup up to this many candidates (DGC_SET_ONE)
constexpr int64_t kQueueFold = 16384;           // k_nth_select emits its replay itself when every k <= this

int64_t payload_layout(int64_t capacity, int vd, int id, int64_t* voff, int64_t* ioff);   // decompress.hip

// One compressed tensor (device table, built on the host).
struct TDesc {
    int64_t n;              // numel
    int64_t off;            // element offset in the flat grad / mmt / vec buffers (multiple of kSeg)
    int64_t seg0, nseg;     // global segments
    int64_t grp0, ngrp;     // global groups
    int64_t k, S, ks, stride;          // num_selects, num_samples, top_k_samples, sample_stride
    int64_t upper_count, lower_count;  // floor(k * upper), ceil(lower * k)
    int64_t samp_off;       // offset of its samples in the flat sample buffer; -1: none / N == S
    int64_t win_off, win_cap;          // its K1 sample window list in the sample buffer (cap 0: none)
    int64_t whist_off;                 // K1's histogram of that window (kWinBins u32, zero at rest)
    int64_t cand_off, cand_cap;        // K5 queue region: min(N, 64k - 1) candidates
    int64_t gpos_off;       // K5 pair slots: 2 x (cand_cap / 2 + 1)
    int64_t idx_base;       // added to the emitted indices (its flat offset in a batch, 0 alone)
    int64_t nv4;            // float4s that K1 streams (n/4 unpadded, ceil(n/4) padded)
    double inv_stride;
    float inv_stride_f;
    int32_t tail;           // the elements [4*nv4, n) are compensated outside K1 (unpadded)
};

struct SelState {
    float t0, t_cur, t_list;
    int32_t branch, iter, recounts, active;
    long long n_cur;       // count at t_cur
    long long limit;       // FIRSTK: emit the first `limit` candidates
    int32_t overflow, done, lower_pending;
    int32_t full_passes, list_spills, epoch;
    int32_t rs_nth;        // RESAMPLE: 1 = nth_element replay (K5), 2 = partial_sort replay (K5b)
    int32_t tie_rule;      // DGC_TIES_*: how the resample chose among boundary ties
    // Deferred momentum masking (DGCSGDMemory.update, dgc/memory.py:72-77): the last
    // call emitted "the first def_limit elements >= def_t" without zeroing them; the
    // next K1, which streams vec and mmt anyway, zeroes them before compensating.
    int32_t def_mode, def_mask_mmt;
    float def_t;
    int32_t win_keys;      // keys K3 read from the K1 sample window list (0: the samples)
    uint32_t win_key;      // the window's key (K1's block 0): its histogram's bin 0
    long long def_limit;
    uint32_t tickets[4];
    uint32_t tk8[9];       // sharded arrival of the count passes (last_block_arrival8)
    uint32_t ce_ticket;    // k_count_emit: groups in ticket order (look-back)
    int32_t ce_fail;       // k_count_emit: a look-back timed out (its emit is not trusted)
    int32_t spec_emitted;  // k_count_emit's first-k payload stands: k_emit skips the tensor
    // Segments whose K1 list overflowed, counted by K1 into slot [epoch & 1] (64
    // shards against atomic contention); k_sel_init reads it and zeroes the other
    // slot for the next call, k_sel_finish advances the epoch.
    uint32_t spill[2][kSpillShards];
    // Samples with key >= key(t_list) that K1 appended to the tensor's window list, in
    // slot [epoch & 1] like spill (the count runs past win_cap when the list overflows).
    uint32_t win_cnt[2];
    unsigned long long lower_cnt[kMaxLower + 1];   // counts at t_1..t_m (multi-threshold pass)
};

// K5s over co-resident workgroups per tensor (k_resample_set): the residency consensus,
// the barrier, the key range and the per-pass histograms. arrive / decide / bar_* /
// broken / mn / mx are reset by sel_init_tensor every call; hist is zero at rest (the
// workspace is zero-filled at init; the workgroups re-zero what they used).
struct SetG {
    uint32_t arrive, decide, bar_count, bar_gen, broken;
    uint32_t gathered;                      // k_emit_set: the tensor's emit workgroups done with its gather
    uint32_t mn, mx;
    uint32_t cnt[kSetGBig];                 // per workgroup: its candidates >= the k-th key
    uint32_t hist0[kSetBins0], hist1[kSetBins1];   // the radix passes' merged histograms
};

// Per-call settings shared by the tensors.
struct SelCfg {
    float upper, lower;         // fl32(compress_upper_bound), fl32(compress_lower_bound)
    int32_t max_iters, resample, masking, vdtype, idtype;
    int32_t update_memory;      // 0: none, 1: zero the emitted slots now, 2: deferred to the next K1
    int32_t tdtype;             // the sparsified tensor's dtype: threshold *= bound rounds to it
    int32_t set_order;          // resample_order = 1: an untied resample emits its set in index order (K5s)
};

// Block tables: prefix arrays [T + 1] of per-tensor workgroup counts for one launch shape.
enum { BT_K1 = 0, BT_FULL, BT_CAP16, BT_CAP4, BT_FULL8, BT_CAP8, BT_SEG, BT_GRP, BT_QUEUE, BT_SAMP, BT_CNT, BT_SET, BT_COUNT };

struct SelWS {
    int32_t T;
    TDesc* td;
    SelState* st;
    RSState* rs;               // [T]: K3 thresholds, then the resample's radix select
    float* thr;                // [T] sampled thresholds
    float* spec;               // [2T] speculative list thresholds (null: none), persistent
    int64_t* starts;           // [T] sample starts of this call
    const float** gptr;        // [T] per-tensor gradient pointers of this call (K1 from a pointer table)
    int64_t* scnt;             // [T] strided sample counts of this call
    float* samples;            // flat sample buffer
    int32_t* bt[BT_COUNT];     // block tables
    int32_t* small;            // tensors whose threshold runs in one workgroup
    uint32_t* seg_lcnt;        // list count at t_list (low 16 bits) | lmax_code (high 16 bits)
    uint32_t* seg_cnt;
    uint32_t* seg_off;         // in-group output offset of each segment's first emitted entry
    uint16_t* lst_off;
    float* lst_val;
    unsigned long long* grp_cnt;
    long long* grp_off;
    unsigned long long* grp_lb;    // k_count_emit's decoupled look-back words, one per group
    uint64_t* queue;           // K5: (|x| key << 32 | j) for the candidates j, ascending index order
    int64_t* cand_idx;         // K5: the candidates' element indices (within the tensor)
    float* cand_val;           // K5: their values (what the gather read; the set path's emit)
    uint32_t* cand_key;        // K5: their |x| keys, dense (the set paths read 4 B per candidate, not 8)
    uint32_t* gpos;            // K5: pair slots of the global-memory partition passes
    NthG* nthg;                // [T] K5: the multi-workgroup global phase's state
    SetG* setg;                // [T] K5s over kSetG workgroups of one launch
    uint32_t* fin_ticket;      // k_nth_select's last-workgroup ticket (zeroed by sel_init_tensor)
    uint32_t* chain;           // k_chain_one's claim / completion / gate words (zeroed by sel_init_tensor)
    int64_t nseg, ngrp;
};

// Candidates the nth_element replay (K5) gathers: torch's CPU topk runs nth_element
// while k * 64 > n (else partial_sort, replayed over vec by K5b), so at most 64k - 1.
__host__ __device__ inline int64_t nth_cand_cap(int64_t numel, int64_t k) {
    const int64_t c = 64 * k - 1;
    return c < numel ? c : numel;
}

// ------------------------------------------------------------------ host layout
// Everything the host derives from the tensor list: the device table image, the
// block tables and the workspace carve. Recomputed on every call (O(T)).
struct TensorIn {
    int64_t n, off, k, S, ks, stride, upper_count, lower_count;
    bool samples;   // reserve a sample buffer (compress); false for a pure selection
};

struct Layout {
    int32_t T = 0;
    int64_t nseg = 0, ngrp = 0, nsamp = 0, ncand = 0, ngpos = 0;
    int64_t max_cand = 0;       // the largest K5 candidate capacity of a tensor
    int64_t max_k = 0;          // the largest num_selects
    int32_t nsmall = 0;
    int32_t nwins = 0;          // tensors with a K1 sample window (their ids follow the small ones)
    int32_t nplain = 0;         // multi-block threshold tasks without a window (k_rs_reset_samples)
    bool adapt_any = false;     // some tensor has N > S (the adaptation loop can run)
    bool tail_any = false;      // some tensor is compensated partly outside K1 (unpadded tail)
    int64_t grid[BT_COUNT] = {};
};

// Capped grids serve the launches that are most likely gated no-ops (the list count
// usually serves), so a small grid keeps their cost down — for a flat bucket, whose
// lists serve in the steady state. A model set's passes run most steps (its synthetic
// thresholds jump), and there a 2048-block cap left the big tensors' passes
// short of HBM rate: 8192 blocks took VGG-16-BN 0.896 -> 0.811 ms, ResNet-50 0.367 ->
// 0.361 ms, 16384 VGG-16-BN 0.816 -> 0.805 ms, ResNet-50 unchanged (same box, tools/ab_lib.sh).
// K5s: the fewest workgroups of a cooperative set (beyond kSetCoopMin candidates) — the
// grid holds max(this, ceil(capacity / kSetCoopMin)) per tensor. 16 per tensor made a
// ResNet-50 step dispatch ~430 workgroups of 1024 threads, and its biggest sets started
// 12-14 us into the launch (tools/k5s_prof.py); DGC_SET_G overrides (2..16).
static uint32_t set_gmin() {
    static const uint32_t g = [] {
        const char* e = std::getenv("DGC_SET_G");
        return (uint32_t)(e ? std::min(std::max(std::atoi(e), 2), kSetG) : kSetGDefault);
    }();
    return g;
}

static inline int64_t bt_blocks(int which, const TDesc& d, int64_t total_seg, int64_t cap_blocks) {
    const int64_t cap = std::max<int64_t>(1, ceil_div(cap_blocks * d.nseg, std::max<int64_t>(1, total_seg)));
    switch (which) {
        case BT_K1: return ceil_div(d.nseg, (int64_t)kSegPerBlock4);
        case BT_FULL: return ceil_div(d.nseg, (int64_t)kSegPerBlock16);
        case BT_CAP16: return std::min(ceil_div(d.nseg, (int64_t)kSegPerBlock16), cap);
        case BT_CAP4: return std::min(ceil_div(d.nseg, (int64_t)kSegPerBlock4), cap);
        case BT_FULL8: return ceil_div(d.nseg, (int64_t)(2 * kSegPerBlock4));
        case BT_CAP8: return std::min(ceil_div(d.nseg, (int64_t)(2 * kSegPerBlock4)), cap);
        case BT_SEG: return ceil_div(d.nseg, (int64_t)kBlock);
        case BT_CNT: return ceil_div(d.nseg, (int64_t)kBlock * kCountSegs);
        case BT_GRP: return ceil_div(d.nseg, (int64_t)(kGroupSegs / kEmitSplit));
        case BT_QUEUE: return ceil_div(d.k, (int64_t)kQueuePerBlock);
        case BT_SET:   // K5s: a resample set holds count(t_cur) <= cand_cap > k candidates
            if (d.k < 1 || d.cand_cap <= d.k) return 0;
            if (d.cand_cap <= kSetCoopMin) return 1;
            return std::min<int64_t>(kSetGBig, std::max<int64_t>(set_gmin(), ceil_div(d.cand_cap, kSetCoopMin)));
        case BT_SAMP: {
            const int64_t cnt = d.samp_off < 0 ? d.n : d.S + 1;
            if (cnt <= kSmallN) return 0;   // one-workgroup threshold (k_rs_small_multi)
            return std::min<int64_t>(512, ceil_div(cnt, (int64_t)kBlock * 16));
        }
    }
    return 0;
}

static void build_layout(const TensorIn* in, int32_t T, bool padded, Layout& L, std::vector<TDesc>& td,
                         std::vector<int32_t> (&bt)[BT_COUNT], std::vector<int32_t>& small) {
    L = Layout{};
    L.T = T;
    td.assign(T, TDesc{});
    small.clear();
    int64_t seg_end = 0, grp = 0, samp = 0, cand = 0, gpos = 0;
    for (int32_t t = 0; t < T; ++t) {
        TDesc& d = td[t];
        d.n = in[t].n;
        d.off = in[t].off;
        d.seg0 = d.off / kSeg;
        d.nseg = ceil_div(d.n, (int64_t)kSeg);
        d.grp0 = grp;
        d.ngrp = ceil_div(d.nseg, (int64_t)kGroupSegs);
        grp += d.ngrp;
        d.k = in[t].k;
        d.S = in[t].S;
        d.ks = in[t].ks;
        d.stride = in[t].stride;
        d.upper_count = in[t].upper_count;
        d.lower_count = in[t].lower_count;
        const bool sampled = d.n != d.S;
        L.adapt_any |= sampled;
        d.samp_off = (sampled && in[t].samples) ? samp : -1;
        if (d.samp_off >= 0) samp += (int64_t)align_up((size_t)(d.S + 1), 64);
        // a window list for the multi-block thresholds; its size cannot depend on ks
        // (dgc_compress_begin lays the workspace out without it)
        d.win_cap = (d.samp_off >= 0 && d.S + 1 > kSmallN) ? std::min<int64_t>(d.S + 1, (d.S + 1) / 16 + 4096) : 0;
        d.win_off = samp;
        samp += (int64_t)align_up((size_t)d.win_cap, 64);
        d.whist_off = samp;
        if (d.win_cap > 0) samp += kWinBins;
        d.cand_off = cand;
        d.cand_cap = nth_cand_cap(d.n, d.k);
        cand += d.cand_cap;
        L.max_cand = std::max(L.max_cand, d.cand_cap);
        L.max_k = std::max(L.max_k, d.k);
        d.gpos_off = gpos;
        gpos += 2 * (d.cand_cap / 2 + 1);
        d.idx_base = T > 1 ? d.off : 0;
        d.nv4 = padded ? ceil_div(d.n, (int64_t)4) : d.n / 4;
        d.tail = (!padded && (d.n & 3)) ? 1 : 0;
        L.tail_any |= d.tail != 0;
        d.inv_stride = 1.0 / (double)(d.stride > 0 ? d.stride : 1);
        d.inv_stride_f = 1.0f / (float)(d.stride > 0 ? d.stride : 1);
        seg_end = std::max(seg_end, d.seg0 + d.nseg);
        const int64_t scnt = sampled ? d.S + 1 : d.n;
        if (scnt <= kSmallN) small.push_back(t);
        else if (!(d.win_cap > 0 && !d.tail)) ++L.nplain;
    }
    L.nseg = seg_end;
    L.ngrp = grp;
    L.nsamp = samp;
    L.ncand = cand;
    L.ngpos = gpos;
    L.nsmall = (int32_t)small.size();
    // the windowed tensors after the small ones: k_rs_small_multi tries their windows
    for (int32_t t = 0; t < T; ++t)
        if (td[t].win_cap > 0 && !td[t].tail) small.push_back(t);
    L.nwins = (int32_t)small.size() - L.nsmall;
    for (int which = 0; which < BT_COUNT; ++which) {
        bt[which].assign(T + 1, 0);
        int64_t acc = 0;
        for (int32_t t = 0; t < T; ++t) {
            bt[which][t] = (int32_t)acc;
            acc += bt_blocks(which, td[t], L.nseg, T > 1 ? kCapBlocksBatch : kCapBlocks);
        }
        bt[which][T] = (int32_t)acc;
        L.grid[which] = acc;
    }
}

static SelWS carve_select(void* base, const Layout& L, size_t* bytes = nullptr) {
    SelWS w{};
    w.T = L.T;
    w.nseg = L.nseg;
    w.ngrp = L.ngrp;
    Carver c(base);
    w.td = c.take<TDesc>(L.T);
    w.st = c.take<SelState>(L.T);
    w.rs = c.take<RSState>(L.T);
    w.thr = c.take<float>(L.T);
    w.spec = c.take<float>(kSpecWords * L.T);
    w.starts = c.take<int64_t>(L.T);
    w.gptr = c.take<const float*>(L.T);
    w.scnt = c.take<int64_t>(L.T);
    for (int which = 0; which < BT_COUNT; ++which) w.bt[which] = c.take<int32_t>(L.T + 1);
    w.small = c.take<int32_t>(L.T);
    w.samples = c.take<float>(L.nsamp);
    w.grp_cnt = c.take<unsigned long long>(L.ngrp);
    w.grp_off = c.take<long long>(L.ngrp);
    w.grp_lb = c.take<unsigned long long>(L.ngrp);
    w.seg_lcnt = c.take<uint32_t>(L.nseg);
    w.seg_cnt = c.take<uint32_t>(L.nseg);
    w.seg_off = c.take<uint32_t>(L.nseg);
    w.lst_off = c.take<uint16_t>(ceil_div(L.nseg, (int64_t)kLstTile) * kLstTile * kCap);
    w.lst_val = c.take<float>(ceil_div(L.nseg, (int64_t)kLstTile) * kLstTile * kCap);
    w.queue = c.take<uint64_t>(L.ncand);
    w.cand_idx = c.take<int64_t>(L.ncand);
    w.cand_val = c.take<float>(L.ncand);
    w.cand_key = c.take<uint32_t>(L.ncand);
    w.gpos = c.take<uint32_t>(L.ngpos);
    w.nthg = c.take<NthG>(L.T);
    w.setg = c.take<SetG>(L.T);
    w.fin_ticket = c.take<uint32_t>(16);
    w.chain = c.take<uint32_t>(kChainWords);
    if (bytes) *bytes = c.bytes();
    return w;
}

// The tables of a one-tensor call, written by one tiny kernel (no host copy).
struct OneTable {
    TDesc d;
    int32_t bt[BT_COUNT][2];
    int64_t start;
};

__global__ void k_put_one(SelWS w, OneTable o) {
    if (threadIdx.x != 0) return;
    w.td[0] = o.d;
    for (int which = 0; which < BT_COUNT; ++which) {
        w.bt[which][0] = o.bt[which][0];
        w.bt[which][1] = o.bt[which][1];
    }
    w.small[0] = 0;
    w.starts[0] = o.start;
    const TDesc& d = o.d;
    w.scnt[0] = d.samp_off < 0 ? d.n : ceil_div(d.n - o.start, d.stride);
}

// Per-call sample starts of a batch (random.randint per tensor, drawn on the host),
// 64 per launch in the kernel arguments; also the sample counts. ptrs: K1 reads tensor
// t's gradient from grad[t] (a pointer table: the parameters' own p.grad tensors, no
// copy into the flat buffer) instead of the flat buffer at its offset.
struct StartChunk {
    int32_t first, count;
    int32_t ptrs, pad;
    int64_t start[64];
    const float* grad[64];
};

__global__ void k_put_starts(SelWS w, StartChunk c) {
    const int i = threadIdx.x;
    if (i >= c.count) return;
    const int t = c.first + i;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    w.starts[t] = c.start[i];
    w.scnt[t] = d.samp_off < 0 ? d.n : ceil_div(d.n - c.start[i], d.stride);
    if (c.ptrs) w.gptr[t] = c.grad[i];
}

// The float4 at element e0 of a gradient of n elements that may end inside it (a
// pointer-table gradient is exactly n floats long): elements past n read as 0.
__device__ __forceinline__ float4 ld_tail4(const float* __restrict__ g, int64_t e0, int64_t n) {
    if (e0 + 3 < n) return ld_nt(reinterpret_cast<const float4*>(g + e0));
    return make_float4(g[e0], e0 + 1 < n ? g[e0 + 1] : 0.f, e0 + 2 < n ? g[e0 + 2] : 0.f, 0.f);
}

// ------------------------------------------------------------------ tile helpers
// Upper bound of a segment's largest |x| key, in 16-bit units: every key < code << 16.
// k_count_lists skips the list of a segment whose code says every |x| < t_cur — at
// 7B most lists hold an entry or two below t_cur, and reading them cost a 128-B line
// per segment. NaN keys give codes above any finite threshold's key (never skipped).
__device__ __forceinline__ uint32_t lmax_code(uint32_t max_key) { return (max_key >> 16) + 1; }
// seg_lcnt packs the list count (<= kSeg) with the code: one 4-B store per segment
__device__ __forceinline__ uint32_t lcnt_pack(uint32_t count, uint32_t code) { return count | (code << 16); }
__device__ __forceinline__ uint32_t lcnt_count(uint32_t v) { return v & 0xFFFFu; }
__device__ __forceinline__ uint32_t tile_max_key(const float (&x)[4], uint32_t valid) {
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if ((valid >> j) & 1u) m = max(m, abs_key(x[j]));
    return m;
}

// Lane holds elements e0..e0+3 of a 256-element tile (e0 = tile base + 4*lane) of a
// tensor whose elements start at v (local indices, n of them).
template <bool ALIGNED>
__device__ __forceinline__ void load_tile(const float* __restrict__ v, int64_t n, int64_t e0, float (&x)[4],
                                          uint32_t& valid) {
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

// Append the lanes' flagged elements (element order 4*lane + j) to a segment list
// (lo / lv: its column, entries kLstTile apart).
__device__ __forceinline__ void list_append(uint32_t p, const float (&x)[4], int tile_off, uint32_t& c,
                                            uint16_t* lo, float* lv, int64_t seg, int64_t ntile) {
    if (__ballot(p != 0)) {
        uint32_t lb, tot;
        wave_prefix4(p, lb, tot);
        uint32_t r = c + lb;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (p & (1u << j)) {
                if (r < (uint32_t)kCap) {
                    lo[lslot(seg, r, ntile)] = (uint16_t)(tile_off + 4 * lane + j);
                    lv[lslot(seg, r, ntile)] = x[j];
                }
                ++r;
            }
        }
        c += tot;
    }
}

// The calling wave's view of local segment ls of a tensor (elements v[0..n)):
// tile u holds elements ls*1024 + 256u + 4*lane + j. All loads are issued before
// any use; 16-B loads when the tensor base is 16-B aligned (a uniform branch).
__device__ __forceinline__ void load_segment(const float* __restrict__ v, int64_t n, int64_t ls,
                                             float (&x)[kSegTiles][4], uint32_t (&valid)[kSegTiles]) {
    const int lane = threadIdx.x & 63;
    if (aligned16(v)) {
#pragma unroll
        for (int u = 0; u < kSegTiles; ++u) load_tile<true>(v, n, ls * kSeg + u * 256 + 4 * lane, x[u], valid[u]);
    } else {
#pragma unroll
        for (int u = 0; u < kSegTiles; ++u) load_tile<false>(v, n, ls * kSeg + u * 256 + 4 * lane, x[u], valid[u]);
    }
}

// Count of |x| >= t over local segment ls of a tensor, re-read by the calling wave.
__device__ uint32_t wave_count_segment(const float* __restrict__ v, int64_t n, int64_t ls, float t) {
    float x[kSegTiles][4];
    uint32_t valid[kSegTiles];
    load_segment(v, n, ls, x, valid);
    uint32_t c = 0;
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) c += __popc(ge_mask(x[u], valid[u], t));
    return wave_sum(c);
}

__device__ __forceinline__ int task(const SelWS& w, int which, int b) { return task_of_block(w.bt[which], w.T, b); }

// The last call's deferred masking for one segment (one wave): zero, in the loaded
// tiles, the elements that call emitted — the first def_limit elements (flat
// order) with |vec| >= def_t, ranked by grp_off + seg_off + in-segment rank. vec is
// unchanged since that emit, so the recount reproduces its choice exactly.
__device__ __forceinline__ void apply_deferred_mask(const SelState& st, const SelWS& w, const TDesc& d,
                                                    int64_t ls, int lane, float4 (&vv)[kSegTiles],
                                                    float4 (&mv)[kSegTiles]) {
    const float dt = st.def_t;
    const long long dlim = st.def_limit;
    const bool mm = st.def_mask_mmt != 0;
    long long rank = w.grp_off[d.grp0 + ls / kGroupSegs] + w.seg_off[d.seg0 + ls];
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) {
        if (rank >= dlim) break;   // wave-uniform
        const int64_t v = ls * (kSeg / 4) + u * 64 + lane;
        const float xo[4] = {vv[u].x, vv[u].y, vv[u].z, vv[u].w};
        const uint32_t pm = ge_mask(xo, v < d.nv4 ? 0xFu : 0u, dt);
        uint32_t lb, tot;
        wave_prefix4(pm, lb, tot);
        long long r = rank + lb;
        float* vf = reinterpret_cast<float*>(&vv[u]);
        float* mf = reinterpret_cast<float*>(&mv[u]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (pm & (1u << j)) {
                if (r < dlim) {
                    vf[j] = 0.f;
                    if (mm) mf[j] = 0.f;
                }
                ++r;
            }
        rank += tot;
    }
}

// Applies a pending deferred masking without compensating (flush before anyone reads
// vec/mmt, and the non-list K1 fallback). One wave per segment.
__global__ void __launch_bounds__(kBlock) k_mask_flush(float* __restrict__ vec_flat, float* __restrict__ mmt_flat,
                                                       SelWS w) {
    const int t = task(w, BT_K1, blockIdx.x);
    const SelState* st = w.st + t;
    if (!st->def_mode) return;
    const TDesc d = w.td[t];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t ls = ((int64_t)blockIdx.x - w.bt[BT_K1][t]) * kSegPerBlock4 + wave;
    if (ls >= d.nseg) return;
    float* vec = vec_flat + d.off;
    float* mmt = st->def_mask_mmt ? mmt_flat + d.off : nullptr;
    const float dt = st->def_t;
    const long long dlim = st->def_limit;
    long long rank = w.grp_off[d.grp0 + ls / kGroupSegs] + w.seg_off[d.seg0 + ls];
    if (rank >= dlim) return;
    float x[kSegTiles][4];
    uint32_t valid[kSegTiles];
    load_segment(vec, d.n, ls, x, valid);
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) {
        const uint32_t pm = ge_mask(x[u], valid[u], dt);
        uint32_t lb, tot;
        wave_prefix4(pm, lb, tot);
        long long r = rank + lb;
        const int64_t e0 = ls * kSeg + u * 256 + 4 * lane;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (pm & (1u << j)) {
                if (r < dlim) {
                    vec[e0 + j] = 0.f;
                    if (mmt) mmt[e0 + j] = 0.f;
                }
                ++r;
            }
        rank += tot;
    }
}

__global__ void k_def_clear(SelWS w) {
    for (int t = threadIdx.x; t < w.T; t += blockDim.x) w.st[t].def_mode = 0;
}

static int mask_flush(float* vec, float* mmt, const Layout& L, const SelWS& w, hipStream_t s) {
    if (L.grid[BT_K1] > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: n too large");
    if (L.grid[BT_K1] > 0) {
        hipLaunchKernelGGL(k_mask_flush, dim3((unsigned)L.grid[BT_K1]), dim3(kBlock), 0, s, vec, mmt, w);
        DGC_LAUNCHED();
    }
    hipLaunchKernelGGL(k_def_clear, dim3(1), dim3(256), 0, s, w);
    DGC_LAUNCHED();
    return DGC_OK;
}

// ------------------------------------------------------------------ K1 with lists
// K1 (compensate + strided sample, see compensate.hip) that also lists every
// element with |vec_new| >= t_list into its segment's list. One wave per segment:
// float4 index = 256*seg + 64*u + lane (u = 0..3), each instruction 1 KB contiguous;
// non-temporal loads and stores. seg_lcnt = exact count at t_list; a segment that
// holds an unpadded scalar tail is marked spilled (re-read when needed).
// ONE (a one-tensor call): the tensor's tables ride in the arguments (ot) — block 0
// writes them into the workspace for the kernels after K1, which replaces a k_put_one
// launch before every K1 (and its wait) — and the sample start in sc.
template <bool NEST, bool ONE>
__global__ void __launch_bounds__(kBlock)
k_compensate_list(const float* __restrict__ g_flat, float* __restrict__ mmt_flat, float* __restrict__ vec_flat,
                  float mom, SelWS w, StartChunk sc, int wt, OneTable ot) {
    const int t = ONE ? 0 : task(w, BT_K1, blockIdx.x);
    const TDesc d = ONE ? ot.d : w.td[t];   // by value: stores below cannot alias it
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t b0 = ONE ? 0 : w.bt[BT_K1][t];   // the tensor's first block
    const int64_t ls = ((int64_t)blockIdx.x - b0) * kSegPerBlock4 + wave;   // local segment
    if (ONE && blockIdx.x == 0 && threadIdx.x == 0) {
        w.td[0] = ot.d;
        for (int which = 0; which < BT_COUNT; ++which) {
            w.bt[which][0] = ot.bt[which][0];
            w.bt[which][1] = ot.bt[which][1];
        }
        w.small[0] = 0;
    }
    // sample starts (and gradient pointers) of the first sc.count tensors ride in the arguments
    const bool arg_start = t < sc.count;
    const float* gsrc = !sc.ptrs ? g_flat + d.off : (arg_start ? sc.grad[t] : w.gptr[t]);
    const float4* g = reinterpret_cast<const float4*>(gsrc);
    float4* mmt = reinterpret_cast<float4*>(mmt_flat + d.off);
    float4* vec = reinterpret_cast<float4*>(vec_flat + d.off);
    const int64_t n4 = d.nv4, n = d.n;
    const float tl = w.spec ? w.spec[kSpecWords * t] : __builtin_huge_valf();
    SelState* st = w.st + t;
    if (blockIdx.x == b0 && threadIdx.x == 0) st->t_list = tl;
    const bool sample = d.samp_off >= 0;
    const int64_t start = !sample ? 0 : (arg_start ? sc.start[t] : w.starts[t]);
    const int64_t scount = !sample ? 0 : (arg_start ? ceil_div(d.n - start, d.stride) : w.scnt[t]);
    if (arg_start && blockIdx.x == b0 && threadIdx.x == 0) {
        w.starts[t] = sc.start[t];
        w.scnt[t] = sample ? scount : d.n;
    }
    float* sout = sample ? w.samples + d.samp_off : nullptr;
    // the sample window list: every sample with key >= the window threshold spec[2] (a
    // prediction of this call's sampled threshold, just below it; the list threshold
    // before the first prediction), inf and NaN too
    float* win = w.samples + d.win_off;
    const float tw = w.spec ? w.spec[kSpecWords * t + 2] : __builtin_huge_valf();
    const uint32_t win_key = abs_key(tw < __builtin_huge_valf() ? tw : tl);
    const bool windowed = sample && d.win_cap > 0;
    uint32_t* win_cnt = &st->win_cnt[st->epoch & 1];
    uint32_t* whist = reinterpret_cast<uint32_t*>(w.samples + d.whist_off);
    if (windowed && blockIdx.x == b0 && threadIdx.x == 0) st->win_key = win_key;
    // waves past the tensor's last segment load nothing and list nothing, but stay for
    // the block barrier of the spill count
    int64_t q0 = 0, r0 = 0;
    if (sample) floor_divmod_fast(ls * kSeg - start, d.stride, d.inv_stride, q0, r0);
    float4 gv[kSegTiles], mv[kSegTiles], vv[kSegTiles];
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) {
        const int64_t v = ls * (kSeg / 4) + u * 64 + lane;
        if (v < n4) {
            gv[u] = sc.ptrs && 4 * v + 3 >= n ? ld_tail4(gsrc, 4 * v, n) : ld_nt(g + v);
            mv[u] = ld_nt(mmt + v);
            vv[u] = ld_nt(vec + v);
        }
    }
    uint32_t c = 0, mk = 0;
    const int64_t seg = d.seg0 + ls;
    uint16_t* lo = w.lst_off;
    float* lv = w.lst_val;
    const int64_t ntile = ceil_div(w.nseg, (int64_t)kLstTile);
    if (st->def_mode && ls < d.nseg) apply_deferred_mask(*st, w, d, ls, lane, vv, mv);
#pragma unroll
    for (int u = 0; u < kSegTiles; ++u) {
        const int64_t v = ls * (kSeg / 4) + u * 64 + lane;
        const bool ok = v < n4;
        float x[4] = {0.f, 0.f, 0.f, 0.f};
        uint32_t valid = 0;
        bool hit = false;   // this lane's sample (at most one per float4: stride >= 4) joins the window
        float hv = 0.f;
        if (ok) {
            x[0] = comp1<NEST, true>(gv[u].x, mv[u].x, vv[u].x, mom);
            x[1] = comp1<NEST, true>(gv[u].y, mv[u].y, vv[u].y, mom);
            x[2] = comp1<NEST, true>(gv[u].z, mv[u].z, vv[u].z, mom);
            x[3] = comp1<NEST, true>(gv[u].w, mv[u].w, vv[u].w, mom);
            st_stream(mmt + v, mv[u], wt);
            st_stream(vec + v, vv[u], wt);
            const int64_t e = 4 * v;
            valid = e + 3 < n ? 0xFu : (e + 2 < n ? 7u : (e + 1 < n ? 3u : (e < n ? 1u : 0u)));
            if (sample) {
                const uint32_t tt = (uint32_t)r0 + 4u * (uint32_t)(u * 64 + lane);
                const uint32_t s32 = (uint32_t)d.stride;
                uint32_t q1, r;
                divmod_u32(tt, s32, d.inv_stride_f, q1, r);
                const uint32_t j = r == 0 ? 0u : s32 - r;
                if (j < 4 && ((valid >> j) & 1u)) {
                    const int64_t qi = q0 + q1 + (r == 0 ? 0 : 1);
                    if (qi >= 0 && qi < scount) {
                        hv = fabsf(x[j]);
                        sout[qi] = hv;
                        hit = windowed && __float_as_uint(hv) >= win_key;
                    }
                }
            }
        }
        const uint64_t hb = __ballot(hit);
        if (hb) {   // wave-uniform and rare (~3 ks of the S samples): one atomic per wave
            const int leader = __ffsll((unsigned long long)hb) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(win_cnt, (uint32_t)__popcll(hb));
            base = __shfl(base, leader);
            const uint32_t pos = base + (uint32_t)__popcll(hb & ((1ull << lane) - 1));
            if (hit && pos < (uint64_t)d.win_cap) win[pos] = hv;
            if (hit) atomicAdd(&whist[win_bin(__float_as_uint(hv), win_key)], 1u);   // (no return value)
        }
        list_append(ge_mask(x, valid, tl), x, u * 256, c, lo, lv, seg, ntile);
        mk = max(mk, tile_max_key(x, valid));
    }
    const bool spilled = c > (uint32_t)kCap;
    mk = wave_max(mk);
    if (lane == 0 && ls < d.nseg) {
        const bool tail = d.tail && ls == d.nseg - 1;   // its scalar tail is compensated outside K1
        w.seg_lcnt[seg] = tail ? lcnt_pack(kCap + 1, 0xFFFFu) : lcnt_pack(c, lmax_code(mk));
    }
    // one atomic per workgroup with a spilled segment (shard by block)
    const uint64_t any = __ballot(spilled);
    __shared__ uint32_t nsp;
    if (threadIdx.x == 0) nsp = 0;
    __syncthreads();
    if (lane == 0 && any) atomicAdd(&nsp, 1u);
    __syncthreads();
    if (threadIdx.x == 0 && nsp) atomicAdd(&st->spill[st->epoch & 1][blockIdx.x % kSpillShards], nsp);
}

__global__ void k_no_lists(SelWS w) {
    for (int t = threadIdx.x; t < w.T; t += blockDim.x) w.st[t].t_list = __builtin_huge_valf();
}

// ------------------------------------------------------------------ state
// Reset tensor t's selection state for this call, by the whole calling workgroup (any
// size): the workgroup that just produced its sampled threshold (k_rs_small_multi, or
// the last workgroup of the final k_rs_hist pass — no launch of its own), or
// k_sel_init for a pure selection (dgc_select, the threshold given).
__device__ void sel_init_tensor(const SelWS& w, int t, int keep_lists) {
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    SelState* st = w.st + t;
    __shared__ uint32_t setg_broken;
    if (threadIdx.x == 0) {   // K5's multi-workgroup barrier and consensus start from zero
        w.nthg[t].bar_count = 0;
        w.nthg[t].bar_gen = 0;
        w.nthg[t].arrive = 0;
        w.nthg[t].decide = 0;
        w.nthg[t].status = 0;
        w.nthg[t].exited = 0;
        w.nthg[t].replayed = 0;
        SetG& sg = w.setg[t];
        setg_broken = sg.broken;
        sg.arrive = sg.decide = sg.bar_count = sg.bar_gen = sg.broken = sg.gathered = 0;
        sg.mn = 0xFFFFFFFFu;
        sg.mx = 0;
        if (t == 0) *w.fin_ticket = 0;
    }
    // k_chain_one's words (k_rs_passes', past kChainOneWords, are zero at rest); one store
    // per thread (every caller runs >= kBlock threads): a strided loop here gave
    // k_rs_small_multi a 320 B/lane scratch frame and doubled its time (15 -> 29 us)
    static_assert(kChainOneWords <= kBlock, "sel_init_tensor: one chain word per thread");
    if (t == 0 && threadIdx.x < kChainOneWords) w.chain[threadIdx.x] = 0;
    __shared__ uint32_t spills;
    if (threadIdx.x == 0) spills = 0;
    __syncthreads();   // the caller's threshold (thr[t]) is written
    if (setg_broken) {
        // a barrier of this tensor's last K5s timed out: its workgroups may have run
        // different numbers of passes, leaving merged-histogram bins they did not re-zero
        // (or re-zeroed before a late add) — restore "zero at rest" for the whole table
        SetG& sg = w.setg[t];
        for (int q = threadIdx.x; q < kSetBins0; q += blockDim.x) sg.hist0[q] = 0;
        for (int q = threadIdx.x; q < kSetBins1; q += blockDim.x) sg.hist1[q] = 0;
    }
    // every load of the reset in flight at once — the epoch, both spill slots, the
    // threshold, the window count: as three dependent round trips they were ~3 us of K3
    const int ep = st->epoch;
    uint32_t sp0 = 0, sp1 = 0;
    if (threadIdx.x < kSpillShards) {
        sp0 = st->spill[0][threadIdx.x];
        sp1 = st->spill[1][threadIdx.x];
    }
    float t0 = 0.f;
    uint32_t win_n = 0;
    if (threadIdx.x == 0) {
        t0 = w.thr[t];
        win_n = w.rs[t].win_n;
    }
    for (int64_t i = threadIdx.x; i < d.ngrp; i += blockDim.x) {
        w.grp_cnt[d.grp0 + i] = 0;
        w.grp_lb[d.grp0 + i] = 0;
    }
    const int e = ep & 1;
    if (threadIdx.x < kSpillShards) {
        const uint32_t v = e ? sp1 : sp0;
        if (v) atomicAdd(&spills, v);
        st->spill[e ^ 1][threadIdx.x] = 0;   // slot of the next call's K1
    }
    if (threadIdx.x == 0) {
        st->win_cnt[e ^ 1] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        st->win_keys = (d.win_cap > 0 && !d.tail) ? (int32_t)win_n : 0;
        st->t0 = t0;
        st->t_cur = t0;
        st->list_spills = keep_lists ? (int32_t)spills : 0;
        // no K1 lists, or too many overflowed lists to be worth serving: one full pass
        if (!keep_lists || (int64_t)spills * kSpillDiv > d.nseg) st->t_list = __builtin_huge_valf();
        st->branch = -1;
        st->n_cur = st->limit = 0;
        st->iter = st->recounts = 0;
        st->active = 1;
        st->overflow = 0;
        st->done = 0;
        st->lower_pending = 0;
        st->full_passes = 0;
        st->rs_nth = 0;
        st->tie_rule = DGC_TIES_NONE;
        for (int i = 0; i < 4; ++i) st->tickets[i] = 0;
        for (int i = 0; i < 9; ++i) st->tk8[i] = 0;
        for (int i = 0; i <= kMaxLower; ++i) st->lower_cnt[i] = 0;
        st->ce_ticket = 0;
        st->ce_fail = 0;
        st->spec_emitted = 0;
    }
}

// Chunked exclusive scan of a[0..m) into out[] by one workgroup; returns the total.
// a[] holds totals accumulated by device atomics: read with agent-scope loads, in
// chunks of kScanReg kept in registers so a chunk's loads are in flight together (a
// loop of dependent loads pays an L2 round trip each); a thread's run of <= kScanReg
// entries is loaded once.
constexpr int kScanReg = 8;
__device__ uint64_t block_scan_array(const unsigned long long* a, long long* out, int64_t m, uint64_t* lds16) {
    const int64_t per = ceil_div(m, (int64_t)blockDim.x);
    const int64_t b = threadIdx.x * per, e = b + per < m ? b + per : m;
    uint64_t v[kScanReg];
    uint64_t local = 0;
    for (int64_t i0 = b; i0 < e; i0 += kScanReg) {
#pragma unroll
        for (int u = 0; u < kScanReg; ++u) v[u] = i0 + u < e ? load_count(&a[i0 + u]) : 0;
#pragma unroll
        for (int u = 0; u < kScanReg; ++u) local += v[u];
    }
    uint64_t total;
    uint64_t run = block_exclusive_scan(local, lds16, &total);
    for (int64_t i0 = b; i0 < e; i0 += kScanReg) {
        if (per > kScanReg) {
#pragma unroll
            for (int u = 0; u < kScanReg; ++u) v[u] = i0 + u < e ? load_count(&a[i0 + u]) : 0;
        }
#pragma unroll
        for (int u = 0; u < kScanReg; ++u)
            if (i0 + u < e) {
                out[i0 + u] = (long long)run;
                run += v[u];
            }
    }
    return total;
}

// One step of the reference's adaptation loop (dgc/compression.py:128-149) on the
// count of the pass that just ran, for tensor t, by the whole calling workgroup (any
// size): the workgroup of the count pass that arrived last for the tensor (no launch
// of its own). With resample (the default) the loop can only lower the threshold until
// the count reaches lower*k, so the first "lower" step hands over to ONE
// multi-threshold pass (k_lower_counts) instead of recounting one threshold per pass;
// without resample the threshold may also rise, and each step is a recount (count
// pass + decide), like the reference. The group totals are other workgroups' device
// atomics of this launch: read with agent-scope loads (last_block_arrival).
__device__ void decide_tensor(const SelWS& w, const SelCfg& p, int t, int spec = 0) {
    SelState* st = w.st + t;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    __shared__ uint64_t lds16[16];
    __shared__ int finished;
    uint64_t local = 0;
    // 8 loads in flight per thread: a 7B tensor has ~6700 groups, 26 per thread of a
    // 256-thread workgroup — one agent-scope round trip each when issued one by one
    const int64_t bd = blockDim.x;
    for (int64_t i0 = threadIdx.x; i0 < d.ngrp; i0 += 8 * bd) {
        uint64_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = i0 + u * bd < d.ngrp ? load_count(&w.grp_cnt[d.grp0 + i0 + u * bd]) : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) local += v[u];
    }
    uint64_t n;
    block_exclusive_scan(local, lds16, &n);
    if (threadIdx.x == 0) {
        if (st->t_cur < st->t_list) {   // a full select pass just re-listed at t_cur
            st->t_list = st->t_cur;
            st->full_passes += 1;
        }
        const long long cnt = (long long)n, k = d.k;
        const bool adapt = d.n > d.S;
        st->n_cur = cnt;
        int done = 1;
        if (!adapt) {
            st->branch = DGC_BRANCH_DIRECT;
            st->limit = cnt < k ? cnt : k;
        } else if (st->iter >= p.max_iters) {
            st->branch = DGC_BRANCH_EXHAUSTED;
            st->limit = cnt < k ? cnt : k;
        } else if (cnt > k) {
            if (cnt > d.upper_count) {
                if (p.resample) {
                    st->branch = DGC_BRANCH_RESAMPLE;
                    // torch's CPU topk: nth_element while k * 64 > candidates (K5), else
                    // partial_sort (K5b) — both replayed exactly
                    st->rs_nth = (cnt < 64 * k && cnt <= d.cand_cap) ? 1 : 2;
                    st->tie_rule = DGC_TIES_EXACT;
                } else {
                    st->t_cur = thr_mul(st->t_cur, p.upper, p.tdtype);
                    done = 0;
                }
            } else {
                st->branch = DGC_BRANCH_TRUNC;
                st->limit = k;
            }
        } else if (cnt < d.lower_count) {
            if (p.resample && st->iter == 0 && p.max_iters <= kMaxLower) {
                st->lower_pending = 1;   // k_lower_counts finds the final threshold in one pass
                done = 2;
            } else {
                st->t_cur = thr_mul(st->t_cur, p.lower, p.tdtype);
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
            // a first-k branch after k_count_emit: its speculative payload is the emit
            if (spec && st->branch != DGC_BRANCH_RESAMPLE && !st->ce_fail) st->spec_emitted = 1;
        } else {
            st->active = 0;
        }
        finished = done;
    }
    __syncthreads();
    if (finished == 1) block_scan_array(w.grp_cnt + d.grp0, w.grp_off + d.grp0, d.ngrp, lds16);
    __syncthreads();
    if (finished != 1)
        for (int64_t i = threadIdx.x; i < d.ngrp; i += blockDim.x) w.grp_cnt[d.grp0 + i] = 0;
}

__global__ void __launch_bounds__(kScanThreads) k_sel_init(SelWS w, int keep_lists) {
    sel_init_tensor(w, blockIdx.x, keep_lists);
}

// ------------------------------------------------------------------ K3 thresholds
// Sample keys of the tensors (or |vec| itself for a direct tensor, N == S).
struct SampleKeys {
    SelWS w;
    const float* vec_flat;
    __device__ __forceinline__ int task(int b) const { return task_of_block(w.bt[BT_SAMP], w.T, b); }
    __device__ __forceinline__ int first_block(int t) const { return w.bt[BT_SAMP][t]; }
    // participating workgroups: all of the task's for the samples; for the window list
    // (~3 ks keys) one per 4096 keys — 512 workgroups over 83k clustered keys paid
    // their histogram flushes on the same few bins and a 512-way arrival per pass
    __device__ __forceinline__ int blocks(int t) const {
        const int all = w.bt[BT_SAMP][t + 1] - w.bt[BT_SAMP][t];
        const uint32_t wn = w.rs[t].win_n;
        return wn ? min(all, (int)((wn + 4095u) / 4096u)) : all;
    }
    // a windowed task whose window k_rs_small_multi selected in one workgroup is done
    __device__ __forceinline__ bool active(int t) const {
        return !(w.td[t].win_cap > 0 && !w.td[t].tail && w.rs[t].small_done);
    }
    __device__ __forceinline__ RSState* state(int t) const { return w.rs + t; }
    __device__ __forceinline__ float* out(int t) const { return w.thr + t; }
    __device__ __forceinline__ uint32_t* chain() const { return w.chain + kChainOneWords; }   // k_rs_passes
    // the final pass's last workgroup: the threshold is known, reset the selection state
    __device__ __forceinline__ void done(int t) const { sel_init_tensor(w, t, 1); }
    template <class F>
    __device__ __forceinline__ void visit(int t, int64_t lb, int64_t nb, F&& f) const {
        const TDesc d = w.td[t];   // by value: stores below cannot alias it
        const uint32_t wn = w.rs[t].win_n;
        if (wn) {
            visit_dense(w.samples + d.win_off, wn, lb, nb, f);
            return;
        }
        const float* x = d.samp_off < 0 ? vec_flat + d.off : w.samples + d.samp_off;
        visit_dense(x, w.scnt[t], lb, nb, f);
    }
};

// Resets the radix state of every multi-block threshold task with its k (top_k_samples)
// and picks its keys. K1 appended every sample with key >= key(t_list) to the tensor's
// window list; when that list is complete (count <= win_cap) and holds >= ks keys,
// the ks-th largest sample is the ks-th largest of the list — every key above it is
// in the list, NaN and inf keys included — so the three passes read the list (~3 ks
// keys in the steady state) instead of the S samples. The result is the same either
// way. An unpadded tail's samples are written outside K1: no list then.
// ks1 > 0: tensor 0's top_k_samples (the one-tensor compress: dgc_compress_begin's
// table was laid out without it, and this saves re-uploading the table).
__device__ __forceinline__ int64_t ks_of(const TDesc& d, int t, int64_t ks1) { return ks1 > 0 && t == 0 ? ks1 : d.ks; }

__global__ void __launch_bounds__(kBlock) k_rs_reset_samples(SelWS w, int64_t ks1) {
    const int t = blockIdx.x;
    if (w.bt[BT_SAMP][t + 1] == w.bt[BT_SAMP][t]) return;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    if (d.win_cap > 0 && !d.tail) return;   // windowed: k_rs_small_multi reset it (or selected its window)
    rs_reset(w.rs + t, (uint64_t)ks_of(d, t, ks1));
}

// One workgroup per small tensor: all three passes from LDS, then the tensor's
// selection state reset (sel_init_tensor). Workgroups nsmall.. take the windowed
// tensors (K1 appended every sample >= the list threshold to a window list): a
// complete window of ks..kSmallN keys is selected the same way, in ONE workgroup, and
// the multi-workgroup passes skip the tensor (small_done) — the ks-th largest sample is
// the ks-th largest of its window (SampleKeys); for VGG-16-BN's big tensors ~3 ks keys,
// where the passes were four launches. A window that does not qualify is left to them.
__global__ void __launch_bounds__(kScanThreads) k_rs_small_multi(SelWS w, const float* vec_flat, int64_t ks1,
                                                                 int32_t nsmall, int32_t use_hist) {
    const int t = w.small[blockIdx.x];
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const uint64_t ks = (uint64_t)ks_of(d, t, ks1);
    if ((int32_t)blockIdx.x >= nsmall) {
        const SelState* st = w.st + t;
        const uint32_t cnt = st->win_cnt[st->epoch & 1];
        const bool complete = cnt >= ks && cnt <= (uint64_t)d.win_cap;
        uint32_t* gh = reinterpret_cast<uint32_t*>(w.samples + d.whist_off);
        bool take = false;
        if (complete) {   // K1's histogram of the window first (it re-zeroes it), then its keys
            if (use_hist)
                take = rs_window_hist_wg(w.samples + d.win_off, cnt, gh, st->win_key, (uint32_t)ks, w.thr + t);
            else
                for (int q = threadIdx.x; q < kWinBins; q += kScanThreads) gh[q] = 0;
            if (!take && cnt <= (uint32_t)kWinMax) {
                rs_window_wg(w.samples + d.win_off, cnt, ks, w.thr + t);
                take = true;
            }
        } else {
            for (int q = threadIdx.x; q < kWinBins; q += kScanThreads) gh[q] = 0;   // zero at rest
        }
        if (!take) {   // the multi-block passes take the task: its reset (their k, and the
            // window's keys instead of the samples when the window is complete)
            rs_reset(w.rs + t, ks);
            if (threadIdx.x == 0) {
                w.rs[t].small_done = 0u;
                w.rs[t].win_n = complete ? cnt : 0u;
            }
            return;
        }
        if (threadIdx.x == 0) {
            w.rs[t].small_done = 1u;
            w.rs[t].win_n = cnt;   // the record's window_keys (sel_init_tensor)
        }
        sel_init_tensor(w, t, 1);
        return;
    }
    const float* x = d.samp_off < 0 ? vec_flat + d.off : w.samples + d.samp_off;
    rs_small_wg(x, w.scnt[t], ks, w.thr + t);
    sel_init_tensor(w, t, 1);
    RS_STAMP(10);
}

// ------------------------------------------------------------------ count passes
#ifdef DGC_K5_PROF
// tools/pass_prof.py: per-workgroup stamps of the last k_count_pass (kind 0) and
// k_lower_counts (kind 1) launch — entry, past the gate, loads done, arrival, end
__device__ unsigned long long g_pass_prof[2][16384][6];
#define PASS_STAMP(k, i) \
    do { if (threadIdx.x == 0 && blockIdx.x < 16384) g_pass_prof[k][blockIdx.x][i] = wall_clock64(); } while (0)
// slot 5: the first iteration's loads arrived (wave 0; the wait is the profiling build's only)
#define PASS_LOADED(k) \
    do { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); PASS_STAMP(k, 5); } while (0)
// tools/es_prof.py: k_emit_wide_t's workgroups — [0] entry, [1] emit: scan done / set:
// its tensor's gather complete, [2] done
__device__ unsigned long long g_es_prof[4096][3];
#define ES_STAMP(i) \
    do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_es_prof[blockIdx.x][i] = wall_clock64(); } while (0)
#else
#define PASS_STAMP(k, i) do { } while (0)
#define PASS_LOADED(k) do { } while (0)
#define ES_STAMP(i) do { } while (0)
#endif
// t_cur >= t_list: counts from the lists, kCountSegs segments per thread (one group
// per workgroup): the list counts of a thread's segments, then their first 8 entries
// (most lists are shorter), are all in flight before any is used — one thread per
// segment paid two dependent round trips per segment in ~13 waves of workgroups at 7B.
// Spilled segments are re-read by the block's waves. One atomic per block into its group;
// the tensor's last workgroup then takes the adaptation step (decide_tensor).
static_assert(kBlock * kCountSegs == kGroupSegs, "k_count_lists: one group per workgroup");
__device__ __forceinline__ void count_lists_body(const float* __restrict__ vec_flat, const SelWS& w, const SelCfg& p,
                                                 int64_t bx) {
    const int t = task(w, BT_CNT, (int)bx);
    const SelState* st = w.st + t;
    PASS_STAMP(0, 0);
    if (!st->active || !(st->t_cur >= st->t_list)) return;
    PASS_STAMP(0, 1);
    const int64_t ntile = ceil_div(w.nseg, (int64_t)kLstTile);
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const float* vec = vec_flat + d.off;
    const float tc = st->t_cur;
    __shared__ int spill[kBlock * kCountSegs];
    __shared__ int nspill;
    __shared__ uint32_t bsum;
    if (threadIdx.x == 0) {
        nspill = 0;
        bsum = 0;
    }
    __syncthreads();
    const int64_t lseg0 = (bx - w.bt[BT_CNT][t]) * kBlock * kCountSegs;
    uint32_t lc[kCountSegs];
    const uint32_t tkey = abs_key(tc);
#pragma unroll
    for (int j = 0; j < kCountSegs; ++j) {
        const int64_t ls = lseg0 + j * kBlock + threadIdx.x;
        const uint32_t v = ls < d.nseg ? w.seg_lcnt[d.seg0 + ls] : 0u;
        // a segment whose every |x| is below t_cur counts 0 without reading its list
        // (or, spilled, its elements)
        lc[j] = ((v >> 16) << 16) <= tkey ? 0u : lcnt_count(v);
    }
    constexpr int kFirst = 8;   // entries loaded up front (one interleaved line)
    float a[kCountSegs][kFirst];
#pragma unroll
    for (int j = 0; j < kCountSegs; ++j) {
        const int64_t sj = d.seg0 + lseg0 + j * kBlock + threadIdx.x;
#pragma unroll
        for (int e = 0; e < kFirst; ++e)
            if ((uint32_t)e < lc[j] && lc[j] <= (uint32_t)kCap) a[j][e] = w.lst_val[lslot(sj, e, ntile)];
    }
    uint32_t ctot = 0;
#pragma unroll
    for (int j = 0; j < kCountSegs; ++j) {
        const int64_t ls = lseg0 + j * kBlock + threadIdx.x;
        if (ls >= d.nseg) continue;
        const int64_t seg = d.seg0 + ls;
        const uint32_t n = lc[j];
        if (n > (uint32_t)kCap) {
            spill[atomicAdd(&nspill, 1)] = j * kBlock + threadIdx.x;
            continue;
        }
        uint32_t c = 0;
#pragma unroll
        for (int e = 0; e < kFirst; ++e) c += (uint32_t)e < n && fabsf(a[j][e]) >= tc;
        // the rest of a longer list, 16 loads in flight at a time
        for (uint32_t e0 = kFirst; e0 < n; e0 += 16) {
            float v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (e0 + q < n) v[q] = w.lst_val[lslot(seg, e0 + q, ntile)];
#pragma unroll
            for (int q = 0; q < 16; ++q) c += e0 + q < n && fabsf(v[q]) >= tc;
        }
        w.seg_cnt[seg] = c;
        ctot += c;
    }
    ctot = wave_sum(ctot);
    if ((threadIdx.x & 63) == 0 && ctot) atomicAdd(&bsum, ctot);
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    for (int q = wave; q < nspill; q += kSegPerBlock4) {
        const int64_t ls2 = lseg0 + spill[q];
        const uint32_t cs = wave_count_segment(vec, d.n, ls2, tc);
        if ((threadIdx.x & 63) == 0) {
            w.seg_cnt[d.seg0 + ls2] = cs;
            if (cs) atomicAdd(&bsum, cs);
        }
    }
    __syncthreads();
    PASS_STAMP(0, 2);
    if (threadIdx.x == 0 && bsum) atomicAdd(&w.grp_cnt[d.grp0 + lseg0 / kGroupSegs], (unsigned long long)bsum);
    PASS_STAMP(0, 3);
    // the tensor's last workgroup takes the adaptation step (no k_decide launch)
    if (last_block_arrival8(w.st[t].tk8, (uint32_t)(bx - w.bt[BT_CNT][t]),
                            (uint32_t)(w.bt[BT_CNT][t + 1] - w.bt[BT_CNT][t])))
        decide_tensor(w, p, t);
    PASS_STAMP(0, 4);
}

__global__ void __launch_bounds__(kBlock)
k_count_lists(const float* __restrict__ vec_flat, SelWS w, SelCfg p) {
    count_lists_body(vec_flat, w, p, blockIdx.x);
}

// t_cur < t_list: full select pass at t_cur — one wave per SUPER segments (kSuper: 16
// float4 loads in flight per lane), re-lists every segment; seg_lcnt = seg_cnt.
// `which` = BT_FULL (one-shot) or BT_CAP16 (grid-stride within the tensor, for a
// launch that is most likely a gated no-op) — BT_K1 / BT_CAP4 for SUPER = 1. The
// tensor's last workgroup then takes the adaptation step (decide_tensor).
template <bool ALIGNED, int SUPER = kSuper>
__device__ __forceinline__ void select_pass_body(const float* __restrict__ vec_flat, const SelWS& w, int which,
                                                 const SelCfg& p, int64_t bx) {
    static_assert(kGroupSegs % (kSegPerBlock4 * SUPER) == 0, "a workgroup's segments lie in one group");
    const int t = task(w, which, (int)bx);
    const SelState* st = w.st + t;
    PASS_STAMP(0, 0);
    if (!st->active || st->t_cur >= st->t_list) return;
    PASS_STAMP(0, 1);
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const float* vec = vec_flat + d.off;
    const float tc = st->t_cur;
    const int64_t ntile = ceil_div(w.nseg, (int64_t)kLstTile);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int kTiles = SUPER * kSegTiles;   // 16 for kSuper
    __shared__ uint32_t wcnt[kSegPerBlock4];
    __shared__ uint32_t wovf[kSegPerBlock4];
    const int64_t nsuper = ceil_div(d.nseg, (int64_t)SUPER);
    const int64_t nb = w.bt[which][t + 1] - w.bt[which][t];
    for (int64_t bi = bx - w.bt[which][t]; bi * kSegPerBlock4 < nsuper; bi += nb) {
        const int64_t sup = bi * kSegPerBlock4 + wave;
        uint32_t ctot = 0, novf = 0;
        if (sup < nsuper) {
            float x[kTiles][4];
            uint32_t valid[kTiles];
#pragma unroll
            for (int u = 0; u < kTiles; ++u)
                load_tile<ALIGNED>(vec, d.n, sup * (SUPER * kSeg) + u * 256 + 4 * lane, x[u], valid[u]);
            PASS_LOADED(0);
#pragma unroll
            for (int sg = 0; sg < SUPER; ++sg) {
                const int64_t ls = sup * SUPER + sg;
                const int64_t seg = d.seg0 + ls;
                uint32_t c = 0;
                uint16_t* lo = w.lst_off;
                float* lv = w.lst_val;
                if (ls < d.nseg) {   // uniform per wave
                    uint32_t mk = 0;
#pragma unroll
                    for (int u = 0; u < kSegTiles; ++u) {
                        list_append(ge_mask(x[sg * kSegTiles + u], valid[sg * kSegTiles + u], tc),
                                    x[sg * kSegTiles + u], u * 256, c, lo, lv, seg, ntile);
                        mk = max(mk, tile_max_key(x[sg * kSegTiles + u], valid[sg * kSegTiles + u]));
                    }
                    mk = wave_max(mk);
                    if (lane == 0) {
                        w.seg_lcnt[seg] = lcnt_pack(c, lmax_code(mk));
                        w.seg_cnt[seg] = c;
                    }
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
            if (s) atomicAdd(&w.grp_cnt[d.grp0 + (bi * kSegPerBlock4 * SUPER) / kGroupSegs], (unsigned long long)s);
            if (o) atomicAdd(&w.st[t].overflow, (int)o);
        }
        __syncthreads();
    }
    PASS_STAMP(0, 2);
    PASS_STAMP(0, 3);
    // the tensor's last workgroup takes the adaptation step (no k_decide launch)
    if (last_block_arrival8(w.st[t].tk8, (uint32_t)(bx - w.bt[which][t]), (uint32_t)nb))
        decide_tensor(w, p, t);
    PASS_STAMP(0, 4);
}

template <bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
k_select_pass(const float* __restrict__ vec_flat, SelWS w, int which, SelCfg p) {
    select_pass_body<ALIGNED>(vec_flat, w, which, p, blockIdx.x);
}

// One count pass as ONE launch: the list counts (the first ncnt workgroups) beside the
// full select pass (the rest) — a tensor takes one of the two (t_cur >= t_list or not),
// so the two run side by side instead of one launch after the other. Only for calls
// whose decide steps cannot leave a tensor active for a recount within the launch (the
// multi-threshold lowering: resample on, max_iters <= kMaxLower — then a decide either
// finishes the tensor or hands it to the lowering), so both gates read one state.
template <bool ALIGNED, int SUPER>
__global__ void __launch_bounds__(kBlock)
k_count_pass(const float* __restrict__ vec_flat, SelWS w, int which, SelCfg p, int ncnt) {
    if ((int)blockIdx.x < ncnt)
        count_lists_body(vec_flat, w, p, blockIdx.x);
    else
        select_pass_body<ALIGNED, SUPER>(vec_flat, w, which, p, (int64_t)blockIdx.x - ncnt);
}

// Counts at t_j = fl32(t_{j-1} * lower), j = 1..max_iters, in ONE pass over vec (the
// reference's "lower" recounts, dgc/compression.py:140-148, all at once). The last
// workgroup of the tensor picks j* = the first j whose count reaches lower*k (else
// max_iters) and arms the count pass + decide at t_{j*}.
template <bool ALIGNED, int SEGS = 1>
__device__ __forceinline__ void lower_counts_body(const float* __restrict__ vec_flat, const SelWS& w,
                                                  const SelCfg& p, int64_t bx) {
    constexpr int kWhich = SEGS == 1 ? BT_CAP4 : BT_CAP8;   // SEGS segments per wave
    const int t = task(w, kWhich, (int)bx);
    SelState* st = w.st + t;
    PASS_STAMP(1, 0);
    if (!st->lower_pending) return;
    PASS_STAMP(1, 1);
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const float* vec = vec_flat + d.off;
    const int m = p.max_iters;
    float th[kMaxLower + 1];
    th[0] = st->t_cur;
#pragma unroll
    for (int j = 1; j <= kMaxLower; ++j) th[j] = thr_mul(th[j - 1], p.lower, p.tdtype);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ uint32_t part[kSegPerBlock4][kMaxLower + 1];
    if (lane == 0)
        for (int j = 1; j <= kMaxLower; ++j) part[wave][j] = 0;
    // A wave per segment, its four tiles loaded before the first compare, then the m
    // thresholds one after the other (a uniform loop), each compare a ballot whose
    // popcount the scalar unit adds (per-lane "c[j] += |x| >= t_j" over all 16 slots
    // behind a divergent |x| >= t_m branch kept the VALU busy ~5 us per workgroup after
    // its loads: tools/pass_prof.py). Four segments per wave (a quarter of the
    // workgroups — 6227 of them take 10 us to dispatch) was slower either way: 22 us per
    // workgroup with per-lane counts, 16 with these.
    const int64_t nb = w.bt[kWhich][t + 1] - w.bt[kWhich][t];
    const int64_t nsup = ceil_div(d.nseg, (int64_t)SEGS);
    constexpr int kT = SEGS * kSegTiles;
    for (int64_t su = (bx - w.bt[kWhich][t]) * kSegPerBlock4 + wave; su < nsup; su += nb * kSegPerBlock4) {
        float xs[kT][4];
        uint32_t vs[kT];
#pragma unroll
        for (int u = 0; u < kT; ++u) load_tile<ALIGNED>(vec, d.n, su * (SEGS * kSeg) + u * 256 + 4 * lane, xs[u], vs[u]);
#pragma unroll
        for (int u = 0; u < kT; ++u)
#pragma unroll
            for (int q = 0; q < 4; ++q) xs[u][q] = ((vs[u] >> q) & 1u) ? fabsf(xs[u][q]) : -1.f;   // (NaN: never >=)
        PASS_LOADED(1);
        float tj = th[0];
        for (int j = 1; j <= m; ++j) {   // uniform
            tj = thr_mul(tj, p.lower, p.tdtype);   // = th[j]
            uint32_t cj = 0;
#pragma unroll
            for (int u = 0; u < kT; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) cj += (uint32_t)__popcll(__ballot(xs[u][q] >= tj));
            if (lane == 0) part[wave][j] += cj;
        }
    }
    __syncthreads();
    PASS_STAMP(1, 2);
    if (threadIdx.x >= 1 && threadIdx.x <= m) {
        const int j = threadIdx.x;
        const uint64_t v = (uint64_t)part[0][j] + part[1][j] + part[2][j] + part[3][j];
        if (v) atomicAdd(&st->lower_cnt[j], (unsigned long long)v);
    }
    PASS_STAMP(1, 3);
    if (!last_block_arrival(&st->tickets[0], (uint32_t)nb)) return;
    if (threadIdx.x < kWave) {
        // the m counts loaded together, one lane each (a loop of dependent agent-scope
        // loads paid an L2 round trip per threshold); j* = the first reaching lower*k
        const int j = lane + 1;
        const bool hit = j <= m && (long long)load_count(&st->lower_cnt[j]) >= d.lower_count;
        const uint64_t hb = __ballot(hit);
        const int js = hb ? __builtin_ctzll(hb) + 1 : m;
        if (threadIdx.x == 0) {
        st->t_cur = th[js];
        st->iter = js;
        st->recounts = js;
        st->overflow = 0;
        st->lower_pending = 0;
        st->active = 1;   // count pass + decide at t_{j*}
        }
    }
    PASS_STAMP(1, 4);
}

template <bool ALIGNED, int SEGS>
__global__ void __launch_bounds__(kBlock)
k_lower_counts(const float* __restrict__ vec_flat, SelWS w, SelCfg p) {
    lower_counts_body<ALIGNED, SEGS>(vec_flat, w, p, blockIdx.x);
}

// The "lower" recounts served by the K1 candidate lists: the counts at the first
// kLowerLists thresholds t_j that are >= t_list, from the complete lists (a spilled
// segment is re-read by a wave). When one of them reaches lower*k, the first such j
// is the reference's j* and k_lower_counts' pass over vec is skipped; otherwise the
// counts are cleared and k_lower_counts recounts every t_j over vec. One thread per
// segment, like k_count_lists.
constexpr int kLowerLists = 4;

__device__ __forceinline__ void lower_lists_body(const float* __restrict__ vec_flat, const SelWS& w, const SelCfg& p,
                                                 int64_t bx) {
    const int t = task(w, BT_SEG, (int)bx);
    SelState* st = w.st + t;
    if (!st->lower_pending) return;
    float th[kLowerLists + 1];
    th[0] = st->t_cur;
#pragma unroll
    for (int j = 1; j <= kLowerLists; ++j) th[j] = thr_mul(th[j - 1], p.lower, p.tdtype);
    const float tl = st->t_list;
    int ms = 0;   // thresholds t_1..t_ms are served by the lists (uniform per tensor)
#pragma unroll
    for (int j = 1; j <= kLowerLists; ++j)
        if (j <= p.max_iters && th[j] >= tl) ms = j;
    if (ms == 0) return;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const float* vec = vec_flat + d.off;
    __shared__ int spill[kBlock];
    __shared__ int nspill;
    __shared__ uint32_t bsum[kLowerLists + 1];
    if (threadIdx.x == 0) nspill = 0;
    if (threadIdx.x <= kLowerLists) bsum[threadIdx.x] = 0;
    __syncthreads();
    const int64_t lseg0 = (bx - w.bt[BT_SEG][t]) * kBlock;
    const int64_t ls = lseg0 + threadIdx.x;
    uint32_t c[kLowerLists + 1];
#pragma unroll
    for (int j = 0; j <= kLowerLists; ++j) c[j] = 0;
    if (ls < d.nseg) {
        const int64_t seg = d.seg0 + ls;
        const uint32_t lc = lcnt_count(w.seg_lcnt[seg]);
        if (lc <= (uint32_t)kCap) {
            const int64_t ntile = ceil_div(w.nseg, (int64_t)kLstTile);
            for (uint32_t e0 = 0; e0 < lc; e0 += 16) {   // 16 loads in flight at a time
                float v[16];
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if (e0 + q < lc) v[q] = w.lst_val[lslot(seg, e0 + q, ntile)];
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    if (e0 + q < lc) {
                        const float a = fabsf(v[q]);
#pragma unroll
                        for (int j = 1; j <= kLowerLists; ++j) c[j] += (j <= ms) && a >= th[j];
                    }
            }
        } else {
            spill[atomicAdd(&nspill, 1)] = threadIdx.x;
        }
    }
#pragma unroll
    for (int j = 1; j <= kLowerLists; ++j) {
        const uint32_t v = wave_sum(c[j]);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&bsum[j], v);
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6;
    for (int q = wave; q < nspill; q += kSegPerBlock4) {
        float x[kSegTiles][4];
        uint32_t valid[kSegTiles];
        load_segment(vec, d.n, lseg0 + spill[q], x, valid);
        for (int j = 1; j <= ms; ++j) {
            uint32_t cs = 0;
#pragma unroll
            for (int u = 0; u < kSegTiles; ++u) cs += __popc(ge_mask(x[u], valid[u], th[j]));
            cs = wave_sum(cs);
            if ((threadIdx.x & 63) == 0 && cs) atomicAdd(&bsum[j], cs);
        }
    }
    __syncthreads();
    if (threadIdx.x >= 1 && threadIdx.x <= ms && bsum[threadIdx.x])
        atomicAdd(&st->lower_cnt[threadIdx.x], (unsigned long long)bsum[threadIdx.x]);
    const uint32_t nb = (uint32_t)(w.bt[BT_SEG][t + 1] - w.bt[BT_SEG][t]);
    if (!last_block_arrival(&st->tickets[2], nb)) return;
    if (threadIdx.x < kWave) {
        // the ms counts loaded together, one lane each (see k_lower_counts)
        const int jl = (int)(threadIdx.x & 63) + 1;
        const bool hit = jl <= ms && (long long)load_count(&st->lower_cnt[jl]) >= d.lower_count;
        const uint64_t hb = __ballot(hit);
        int js = hb ? __builtin_ctzll(hb) + 1 : 0;
        if (threadIdx.x == 0) {
        // every t_j served and none reaches lower*k: t_(max_iters), as k_lower_counts picks
        if (!js && ms == p.max_iters) js = ms;
        if (js) {
            st->t_cur = th[js];
            st->iter = js;
            st->recounts = js;
            st->overflow = 0;
            st->lower_pending = 0;
            st->active = 1;   // count pass + decide at t_{j*}
        } else {
            for (int j = 1; j <= ms; ++j) st->lower_cnt[j] = 0;   // k_lower_counts recounts every t_j
        }
        }
    }
}

__global__ void __launch_bounds__(kBlock)
k_lower_lists(const float* __restrict__ vec_flat, SelWS w, SelCfg p) {
    lower_lists_body(vec_flat, w, p, blockIdx.x);
}

// ------------------------------------------------------------------ emit
struct EmitOut {
    float* vec;          // flat; null: leave vec untouched (pure selection)
    float* mmt;          // flat; null: no momentum masking
    void* values;
    void* indices;
    int32_t vdtype, idtype;
    uint64_t* queue;     // non-null: K5 candidate gather (queue[pos] = key << 32 | pos, cand[pos] = index)
    int64_t* cand;
    int32_t defer;       // first-k branches: leave vec/mmt to the next K1 (record seg_off instead)
    float* cval;         // the K5 gather: cval[pos] = the candidate's value (null: not kept)
    uint32_t* ckey;      //   and ckey[pos] = its key
    int32_t no_queue;    // the gather leaves queue[] unwritten (k_nth_select rebuilds it from ckey)
};

// Entries a tensor emits: the first `limit` candidates, or k after a resample.
__device__ __forceinline__ long long final_count(const SelState& s, int64_t k) {
    return s.branch == DGC_BRANCH_RESAMPLE ? (long long)k : s.limit;
}

// Output position of a tensor's first entry: the entries of the tensors before it.
// The payload position of tensor t's first entry: the final counts of the tensors
// before it, summed by one wave (all loads in flight at once — a serial loop over 50
// tensors was 50 dependent round trips). Call from a whole wave; every lane gets it.
__device__ __forceinline__ long long out_base(const SelWS& w, int t) {
    long long b = 0;
    for (int u0 = 0; u0 < t; u0 += kWave) {
        const int u = u0 + (int)(threadIdx.x & 63);
        b += u < t ? final_count(w.st[u], w.td[u].k) : 0;
    }
    return wave_sum(b);
}

// pos: output slot; li: the element's index within its tensor (d.off + li in the flat buffers).
__device__ __forceinline__ void emit_one(const EmitOut& o, const TDesc& d, long long pos, int64_t li, float x,
                                         bool mask_now = true) {
    if (o.queue) {
        if (!o.no_queue) o.queue[d.cand_off + pos] = ((uint64_t)abs_key(x) << 32) | (uint64_t)(uint32_t)pos;
        o.cand[d.cand_off + pos] = li;
        if (o.cval) {
            o.cval[d.cand_off + pos] = x;
            o.ckey[d.cand_off + pos] = abs_key(x);
        }
        return;
    }
    store_value(o.values, pos, x, o.vdtype);
    store_index(o.indices, pos, d.idx_base + li, o.idtype);
    if (!mask_now) return;
    // scattered 4-B writes, one per 128-B line: non-temporal (no L2 allocation)
    if (o.vec) __builtin_nontemporal_store(0.f, o.vec + d.off + li);
    if (o.mmt) __builtin_nontemporal_store(0.f, o.mmt + d.off + li);
}

// Wave-cooperative emit of one spilled segment (local ls) from its elements in
// registers (xs / vs: load_segment's).
// FIRSTK: positions base + rank for |x| >= t, kept while < limit.
__device__ __forceinline__ void emit_segment_firstk(const float (&xs)[kSegTiles][4], const uint32_t (&vs)[kSegTiles],
                                                    const TDesc& d, int64_t ls, long long base, long long limit,
                                                    long long obase, float t, const EmitOut& o, bool mask_now) {
    const int lane = threadIdx.x & 63;
    uint32_t run = 0;
#pragma unroll
    for (int tile = 0; tile < kSegTiles; ++tile) {
        const float(&x)[4] = xs[tile];
        const int64_t e0 = ls * kSeg + tile * 256 + 4 * lane;
        const uint32_t pm = ge_mask(x, vs[tile], t);
        if (__ballot(pm != 0)) {
            uint32_t lb, tot;
            wave_prefix4(pm, lb, tot);
            uint32_t r = run + lb;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (pm & (1u << j)) {
                    const long long pos = base + r;
                    if (pos < limit) emit_one(o, d, obase + pos, e0 + j, x[j], mask_now);
                    ++r;
                }
            run += tot;
        }
    }
}

// ... re-reading vec. (Two segments per call with both loads in flight made no
// difference to ResNet-50's emit, whose spilled small tensors end ~17 us into the launch:
// tools/es_prof.py.)
__device__ __forceinline__ void emit_reread_firstk(const float* __restrict__ vec, const TDesc& d, int64_t ls,
                                                   long long base, long long limit, long long obase, float t,
                                                   const EmitOut& o, bool mask_now) {
    float xs[kSegTiles][4];
    uint32_t vs[kSegTiles];
    load_segment(vec, d.n, ls, xs, vs);
    emit_segment_firstk(xs, vs, d, ls, base, limit, obase, t, o, mask_now);
}


// kEmitSplit workgroups of kEmitSegs threads per group of kGroupSegs segments, one
// thread per segment of its quarter. In-group offsets: the quarter's exclusive scan
// plus the counts of the group's earlier quarters (read by the same threads, packed
// into the high half of the one 64-bit scan). Then
//   short lists (<= kEmitShort entries, the common case once the list threshold
//   tracks the selection): the thread emits its own segment, sequentially — its list
//   loads go out before the scan;
//   longer lists: wave per segment — kCap == 64 list slots, lane l takes entry l (one
//   coalesced load per list), ballot ranks give the positions, kEmitBatch lists in
//   flight per wave;
//   spilled segments (> kCap entries): one wave re-reads the 1024 elements.
// o.queue == null: the payload (every branch but a K5 resample, which k_emit_queue
// writes). o.queue != null: K5's candidate gather — every element >= t_cur, ascending
// (the reference's `indices` before its resample topk), only when K5 serves the tensor.
constexpr int kEmitSegs = kGroupSegs / kEmitSplit;   // segments per workgroup (a quarter group)
constexpr int kEmitBatch = 16;
constexpr int kEmitShort = 16;                  // lists up to this long: a thread emits its segment
constexpr uint32_t kEmitSkip = 0xFFFFFFFFu;
static_assert(kCap == kWave, "wave-per-list emission needs kCap == wavefront width");

__device__ __forceinline__ void emit_body(const float* __restrict__ vec_flat, const SelWS& w, const EmitOut& oa,
                                          int64_t bx) {
    const int t = task(w, BT_GRP, (int)bx);
    const SelState* st = w.st + t;
    if (st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 2) return;   // K5b emits it
    if (st->spec_emitted) return;                                        // k_count_emit did
    const bool k5 = st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 1;
    // oa.queue set: the K5 tensors gather their candidates into the queue and the
    // others emit their payload in the same launch; unset: the K5 tensors are skipped
    if (k5 && !oa.queue) return;
    EmitOut o = oa;
    if (!k5) o.queue = nullptr;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    // first-k branches of an engine that defers: the next K1 zeroes what this emits
    const bool defer_here = o.defer && !k5 && !d.tail;
    const float* vec = vec_flat + d.off;
    const int64_t lb = bx - w.bt[BT_GRP][t];
    const int64_t lg = lb / kEmitSplit;                      // group within the tensor
    const int sub = (int)(lb % kEmitSplit);                  // its quarter
    const int64_t g = d.grp0 + lg;
    const int64_t lseg0 = lg * kGroupSegs + (int64_t)sub * kEmitSegs;   // first segment of the quarter
    __shared__ uint32_t off_a[kEmitSegs], lcn[kEmitSegs];
    __shared__ uint64_t lds16[16];
    __shared__ long long obase_s;
    if (threadIdx.x < kWave) {
        const long long b = k5 ? 0 : out_base(w, t);
        if (threadIdx.x == 0) obase_s = b;
    }
    const long long limit = k5 ? st->n_cur : st->limit;
    const long long ga = w.grp_off[g];
    const float tc = st->t_cur;
    {
        // thread jq <-> segment jq of the quarter, plus the earlier quarters' counts at
        // the same position
        const int jq = (int)threadIdx.x;
        const int64_t ls = lseg0 + jq;
        uint32_t ca = 0, lc = 0, pa = 0;
        if (ls < d.nseg) {
            const int64_t seg = d.seg0 + ls;
            ca = w.seg_cnt[seg];
            lc = lcnt_count(w.seg_lcnt[seg]);
        }
#pragma unroll
        for (int q = 0; q < kEmitSplit - 1; ++q) {   // the same position in the group's earlier
            if (q < sub) {                             // quarters (loads in flight together)
                const int64_t seg = d.seg0 + lg * kGroupSegs + (int64_t)q * kEmitSegs + threadIdx.x;
                pa += w.seg_cnt[seg];
            }
        }
        // (a list with nothing at the current threshold is not read: most of them at 1e-4)
        const bool short_list = ls < d.nseg && ca > 0 && lc <= (uint32_t)kEmitShort;
        float v[kEmitShort];
        uint16_t e[kEmitShort];
        if (short_list) {
            const int64_t ntile = ceil_div(w.nseg, (int64_t)kLstTile);
#pragma unroll
            for (int q = 0; q < kEmitShort; ++q)
                if ((uint32_t)q < lc) {
                    v[q] = w.lst_val[lslot(d.seg0 + ls, q, ntile)];
                    e[q] = w.lst_off[lslot(d.seg0 + ls, q, ntile)];
                }
        }
        // (earlier quarters' total << 32) | this quarter's counts: one scan gives both
        uint64_t tot;
        const uint64_t ra = block_exclusive_scan(((uint64_t)pa << 32) | ca, lds16, &tot);
        const uint32_t oa = (uint32_t)(tot >> 32) + (uint32_t)ra;
        const bool work = ca > 0 && ga + oa < limit;
        if (defer_here && ls < d.nseg) w.seg_off[d.seg0 + ls] = oa;
        off_a[jq] = oa;
        lcn[jq] = (work && !short_list) ? lc : kEmitSkip;
        __syncthreads();   // obase_s
        if (work && short_list) {   // the first `limit` entries >= tc, in index order
            const long long ob0 = obase_s;
            long long pos = ga + oa;
#pragma unroll
            for (int j = 0; j < kEmitShort; ++j)
                if ((uint32_t)j < lc && fabsf(v[j]) >= tc) {
                    if (pos < limit) emit_one(o, d, ob0 + pos, ls * kSeg + e[j], v[j], !defer_here);
                    ++pos;
                }
        }
    }
    __syncthreads();
    const long long obase = obase_s;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    // which of the wave's segments are left to it (longer lists) and which spilled:
    // one LDS read and two ballots, so a wave with nothing left skips
    constexpr int kWaveSegs = kEmitSegs / (kEmitSegs / kWave);   // 64: one ballot covers them
    const int jw = wv * kWaveSegs;
    const uint32_t Lme = lane < kWaveSegs ? lcn[jw + lane] : kEmitSkip;
    uint64_t todo = __ballot(Lme != kEmitSkip && Lme <= (uint32_t)kCap);
    uint64_t spilled = __ballot(Lme != kEmitSkip && Lme > (uint32_t)kCap);
    for (int b0 = 0; b0 < kWaveSegs; b0 += kEmitBatch) {
        if (!((todo >> b0) & ((1ull << kEmitBatch) - 1))) continue;   // nothing in this batch
        const int j0 = jw + b0;
        float x[kEmitBatch];
        uint32_t e[kEmitBatch];
#pragma unroll
        for (int q = 0; q < kEmitBatch; ++q) {   // all list loads issued first
            const uint32_t L = lcn[j0 + q];
            x[q] = 0.f;
            e[q] = 0;
            if (L <= (uint32_t)kCap && (uint32_t)lane < L) {
                const int64_t slot = lslot(d.seg0 + lseg0 + j0 + q, lane, ceil_div(w.nseg, (int64_t)kLstTile));
                x[q] = w.lst_val[slot];
                e[q] = w.lst_off[slot];
            }
        }
#pragma unroll
        for (int q = 0; q < kEmitBatch; ++q) {
            const uint32_t L = lcn[j0 + q];
            if (L == kEmitSkip || L > (uint32_t)kCap) continue;
            const int64_t ls = lseg0 + j0 + q;
            const long long ba = ga + off_a[j0 + q];
            const bool sel = (uint32_t)lane < L && fabsf(x[q]) >= tc;
            const uint64_t m = __ballot(sel);
            const long long pos = ba + __popcll(m & lt);
            if (sel && pos < limit) emit_one(o, d, obase + pos, ls * kSeg + e[q], x[q], !defer_here);
        }
    }
    while (spilled) {   // rare: one wave re-reads the segment's 1024 elements
        const int j = jw + __builtin_ctzll(spilled);
        spilled &= spilled - 1;
        emit_reread_firstk(vec, d, lseg0 + j, ga + off_a[j], limit, obase, tc, o, !defer_here);
    }
}

__global__ void __launch_bounds__(kEmitSegs)
k_emit(const float* __restrict__ vec_flat, SelWS w, EmitOut oa) {
    emit_body(vec_flat, w, oa, blockIdx.x);
}

// One-tensor DGC_SYNC_DEVICE selections with the lowering shortcut (the flat bucket):
// the lowering from the lists, the lowering over vec and the count at the lowered
// threshold from the lists — three launches that are gated no-ops in the steady state —
// in ONE launch. The two full select passes and the emit stay launches of their own:
// chained, their HBM-bound bodies ran at the combined kernel's 2 waves per SIMD
// (177 VGPRs) and a step whose lists missed took 0.43 ms longer (flat-1B, same box). When
// every tensor is decided (the steady state: the first count's decide) every workgroup
// returns at once. Otherwise the phases run in order
// over virtual blocks that workgroups claim from an atomic counter; each phase's gate is
// decided once, by the first workgroup to reach it, from the state the phases before
// left; a workgroup waits for a phase's completion count (chain_phase_end: one L2
// write-back per XCD that wrote, an acquire per workgroup) before the next phase. Only
// running workgroups claim blocks, so nothing assumes the grid co-resident.
constexpr int kChainPhases = 3;
enum { CH_CLAIM = 0, CH_GATE = kChainPhases };   // words of the first line; then a ChainPhase each
static_assert(32 + kChainPhases * 32 <= kChainOneWords, "SelWS::chain words");

template <bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
k_chain_one(const float* __restrict__ vec_flat, SelWS w, SelCfg p) {
    uint32_t* cc = w.chain;
    __shared__ uint32_t s_u;
    bool open = false;   // a tensor still adapting (every phase below gates on that)
    for (int t = threadIdx.x; !open && t < w.T; t += blockDim.x) open = !w.st[t].done;
    if (!__syncthreads_or(open)) return;   // uniform: the steady state
    for (int ph = 0; ph < kChainPhases; ++ph) {
        // does any tensor need the phase
        bool any = false;
        for (int t = threadIdx.x; !any && t < w.T; t += blockDim.x) {
            const SelState& u = w.st[t];
            any = ph < 2 ? u.lower_pending != 0 : (u.active && u.t_cur >= u.t_list);
        }
        any = __syncthreads_or(any);   // (also: s_u is free again)
        if (threadIdx.x == 0) {
            uint32_t gate = __hip_atomic_load(&cc[CH_GATE + ph], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (gate == 0) {
                const uint32_t want = any ? 2u : 1u;
                const uint32_t prev = atomicCAS(&cc[CH_GATE + ph], 0u, want);
                gate = prev == 0u ? want : prev;
            }
            s_u = gate;
        }
        __syncthreads();
        if (s_u != 2u) continue;   // uniform
        const int which = ph == 0 ? BT_SEG : ph == 1 ? BT_CAP4 : BT_CNT;
        const uint32_t nvb = (uint32_t)w.bt[which][w.T];
        uint32_t mine = 0;
        for (;;) {
            __syncthreads();
            if (threadIdx.x == 0) s_u = atomicAdd(&cc[CH_CLAIM + ph], 1u);
            __syncthreads();
            const uint32_t vb = s_u;
            if (vb >= nvb) break;   // uniform
            if (ph == 0) lower_lists_body(vec_flat, w, p, vb);
            else if (ph == 1) lower_counts_body<ALIGNED>(vec_flat, w, p, vb);
            else count_lists_body(vec_flat, w, p, vb);
            ++mine;
        }
        chain_phase_end(reinterpret_cast<ChainPhase*>(cc + 32) + ph, mine, nvb);
    }
}



__device__ __forceinline__ void resample_set_block(const float* __restrict__ vec_flat, const SelWS& w,
                                                   const EmitOut& o, int bx, int64_t one_max, uint32_t gmin,
                                                   bool wait);   // K5s, below

// The few groups of a model gradient set: kEmitSplit workgroups of kGroupSegs threads
// per group, each scanning the whole group (thread per segment) and emitting its
// quarter with 16 waves of 16 segments — one list batch per wave, every list by a
// wave. More waves per quarter beat k_emit's short-list threads there (measured on
// ResNet-50: 12 vs 15 us per launch).
//
// SET (k_emit_set): the emit and k_resample_set in ONE launch. The workgroups from ngb
// on are the sets' (resample_set_block); an emit workgroup that gathered a resampled
// tensor's candidates releases its stores and counts itself in the tensor's
// SetG::gathered, and the tensor's sets start once all of its emit workgroups have —
// beside the other tensors' emit, one launch boundary fewer. The emit workgroups come
// first in the grid and never wait, so a waiting set only holds a slot the emit does
// not need (ResNet-50's whole grid, ~220 workgroups of 1024 threads, is resident at
// once on 256 CUs; VGG-16-BN's ~680 against 512 slots, ~150 of them sets).
// Returns true when the workgroup gathered a resampled tensor's candidates.
__device__ __forceinline__ bool emit_wide_part(const float* __restrict__ vec_flat, const SelWS& w, const EmitOut& oa,
                                               int bx) {
    const int t = task(w, BT_GRP, bx);
    const SelState* st = w.st + t;
    if (st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 2) return false;   // K5b emits it
    if (st->spec_emitted) return false;                                        // k_count_emit did
    const bool k5 = st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 1;
    // oa.queue set: the K5 tensors gather their candidates into the queue and the
    // others emit their payload in the same launch; unset: the K5 tensors are skipped
    if (k5 && !oa.queue) return false;
    EmitOut o = oa;
    if (!k5) o.queue = nullptr;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    // first-k branches of an engine that defers: the next K1 zeroes what this emits
    const bool defer_here = o.defer && !k5 && !d.tail;
    const float* vec = vec_flat + d.off;
    const int64_t lb = (int64_t)bx - w.bt[BT_GRP][t];
    constexpr int split = kEmitSplit;
    const int64_t lg = lb / split;                           // group within the tensor
    const int sub = (int)(lb % split);                       // its share this workgroup emits
    const int64_t g = d.grp0 + lg;
    const int64_t lseg0 = lg * kGroupSegs;
    __shared__ uint32_t off_a[kGroupSegs], lcn[kGroupSegs];
    __shared__ uint64_t lds16[16];
    __shared__ long long obase_s;
    if (threadIdx.x < kWave) {
        const long long b = k5 ? 0 : out_base(w, t);
        if (threadIdx.x == 0) obase_s = b;
    }
    const long long limit = k5 ? st->n_cur : st->limit;
    const long long ga = w.grp_off[g];
    {
        const int64_t ls = lseg0 + threadIdx.x;
        uint32_t ca = 0, lc = 0;
        if (ls < d.nseg) {
            const int64_t seg = d.seg0 + ls;
            ca = w.seg_cnt[seg];
            lc = lcnt_count(w.seg_lcnt[seg]);
        }
        uint64_t tot;
        const uint32_t oa = (uint32_t)block_exclusive_scan((uint64_t)ca, lds16, &tot);
        const bool work = ca > 0 && ga + oa < limit;
        if (defer_here && ls < d.nseg && (int)threadIdx.x / (kGroupSegs / split) == sub)
            w.seg_off[d.seg0 + ls] = oa;
        off_a[threadIdx.x] = oa;
        lcn[threadIdx.x] = work ? lc : kEmitSkip;
    }
    __syncthreads();
    ES_STAMP(1);
    const long long obase = obase_s;
    const float tc = st->t_cur;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t lt = lanemask_lt();
    constexpr int wave_segs = kGroupSegs / split / (kGroupSegs / kWave);
    static_assert(wave_segs % kEmitBatch == 0, "whole batches per wave");
    const int jw = sub * (kGroupSegs / split) + wv * wave_segs;
    for (int j0 = jw; j0 < jw + wave_segs; j0 += kEmitBatch) {
        float x[kEmitBatch];
        uint32_t e[kEmitBatch];
#pragma unroll
        for (int q = 0; q < kEmitBatch; ++q) {   // all list loads issued first
            const uint32_t L = lcn[j0 + q];
            x[q] = 0.f;
            e[q] = 0;
            if (L <= (uint32_t)kCap && (uint32_t)lane < L) {
                const int64_t slot = lslot(d.seg0 + lseg0 + j0 + q, lane, ceil_div(w.nseg, (int64_t)kLstTile));
                x[q] = w.lst_val[slot];
                e[q] = w.lst_off[slot];
            }
        }
        uint32_t spilled = 0;   // (re-read after the batch: a call inside kept the loop rolled)
#pragma unroll
        for (int q = 0; q < kEmitBatch; ++q) {
            const uint32_t L = lcn[j0 + q];
            if (L == kEmitSkip) continue;
            const int64_t ls = lseg0 + j0 + q;
            const long long ba = ga + off_a[j0 + q];
            if (L > (uint32_t)kCap) {
                spilled |= 1u << q;
                continue;
            }
            const bool sel = (uint32_t)lane < L && fabsf(x[q]) >= tc;
            const uint64_t m = __ballot(sel);
            const long long pos = ba + __popcll(m & lt);
            if (sel && pos < limit) emit_one(o, d, obase + pos, ls * kSeg + e[q], x[q], !defer_here);
        }
        while (spilled) {   // rare: the wave re-reads the segment's 1024 elements
            const int q = __builtin_ctz(spilled);
            spilled &= spilled - 1;
            emit_reread_firstk(vec, d, lseg0 + j0 + q, ga + off_a[j0 + q], limit, obase, tc, o, !defer_here);
        }
    }
    return k5;
}

template <bool SET>
__global__ void __launch_bounds__(kGroupSegs)
k_emit_wide_t(const float* __restrict__ vec_flat, SelWS w, EmitOut oa, EmitOut os, int64_t one_max, uint32_t gmin,
              int32_t ngb) {
    const int bx = (int)blockIdx.x;
    ES_STAMP(0);
    if (SET && bx >= ngb) {
        resample_set_block(vec_flat, w, os, bx - ngb, one_max, gmin, true);
    } else if (emit_wide_part(vec_flat, w, oa, bx) && SET) {   // uniform per workgroup
        const int t = task(w, BT_GRP, bx);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(&w.setg[t].gathered, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    ES_STAMP(2);
}

// The first count pass of a ONE-tensor call whose lists serve t_cur (the flat
// bucket's steady state), fused with a speculative first-k emit: k_count_lists and
// k_emit read the same list lines one after the other (flat-1B: 32 + 57 us, 7B:
// 112 + 132 us). One workgroup per group, in ticket order; a thread counts four
// consecutive segments, whose list entries e share one 16-B word of a 128-B line.
// The group's offset comes from a decoupled look-back over the earlier groups' words
// (aggregate, then inclusive prefix; a group only waits for groups that took their
// ticket before it, so all of them are running). Every entry >= t_cur at a position
// < k is written: exactly the payload of every first-k branch (ok, trunc, direct,
// exhausted: the first min(count, k)). When decide picks one, spec_emitted makes
// k_emit skip the tensor; otherwise (resample, lower) the later passes emit again
// over it. Host-gated to calls whose emit would not mask (deferred or pure selection)
// and whose payload starts at slot 0 (one tensor).
constexpr unsigned long long kLbAgg = 1ull << 62, kLbPre = 1ull << 63, kLbVal = kLbAgg - 1;
constexpr int kLbSpin = 1 << 22;   // polls (with s_sleep) before a look-back gives up: ~seconds
constexpr int kCeStage = 2048;     // entries a group stages in LDS for coalesced payload writes
#ifdef DGC_K5_PROF
__device__ unsigned long long g_ce_prof[2048][6];   // tools/ce_prof.py: per-group phase stamps
#define CE_STAMP(i) do { if (threadIdx.x == 0 && lg < 2048) g_ce_prof[lg][i] = wall_clock64(); } while (0)
#else
#define CE_STAMP(i) do { } while (0)
#endif

__device__ __forceinline__ void count_emit_body(const float* __restrict__ vec_flat, const SelWS& w, const SelCfg& p,
                                                const EmitOut& o) {
    static_assert(kBlock * kCountSegs == kGroupSegs && kCountSegs == kLstTile, "k_count_emit layout");
    SelState* st = w.st;
    if (!st->active || !(st->t_cur >= st->t_list)) return;
    const TDesc d = w.td[0];   // by value: stores below cannot alias it
    const float* vec = vec_flat + d.off;
    const float tc = st->t_cur;
    const uint32_t tkey = abs_key(tc);
    const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
    __shared__ uint32_t lg_s;
    __shared__ int nspill;
    __shared__ int spill[kGroupSegs];
    __shared__ uint32_t spill_cnt[kGroupSegs];   // a spilled segment's count, then its offset
    __shared__ uint64_t lds16[16];
    __shared__ unsigned long long prefix_s;
    __shared__ float stage_v[kCeStage];
    __shared__ uint32_t stage_i[kCeStage];
    if (tid == 0) {
        lg_s = atomicAdd(&st->ce_ticket, 1u);
        nspill = 0;
    }
    __syncthreads();
    const int64_t lg = lg_s;
    CE_STAMP(0);
    const int64_t ls0 = lg * kGroupSegs + kCountSegs * tid;   // this thread's 4 segments
    const int64_t seg0 = d.seg0 + ls0;                        // a multiple of 4 (one tensor: seg0 = 0)
    uint32_t n[kCountSegs], c[kCountSegs], lc[kCountSegs];
    if (ls0 + 3 < d.nseg) {   // one 16-B load
        const uint4 u = *reinterpret_cast<const uint4*>(w.seg_lcnt + seg0);
        lc[0] = u.x; lc[1] = u.y; lc[2] = u.z; lc[3] = u.w;
    } else {
#pragma unroll
        for (int q = 0; q < kCountSegs; ++q) lc[q] = ls0 + q < d.nseg ? w.seg_lcnt[seg0 + q] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kCountSegs; ++q) {
        n[q] = ((lc[q] >> 16) << 16) <= tkey ? 0u : lcnt_count(lc[q]);   // every |x| < t_cur: nothing
        c[q] = 0;
    }
    uint32_t nmax = 0;   // the longest complete list of the four
#pragma unroll
    for (int q = 0; q < kCountSegs; ++q)
        if (n[q] <= (uint32_t)kCap) nmax = max(nmax, n[q]);
    constexpr int kFirst = 8;   // entries 0..7: the four lists' share of one 128-B line
    const int64_t ntile = ceil_div(w.nseg, (int64_t)kLstTile);
    const float* lv = w.lst_val;
    const uint16_t* lo = w.lst_off;
    // The emit re-reads the entries (from L2) rather than holding them across the scan
    // and look-back: held, with their offsets, they took the kernel to 145 VGPRs, 3 waves
    // per SIMD, and 768 of flat-1B's 977 groups resident — the rest started up to 90 us
    // late (tools/ce_prof.py); re-read it runs at 103 VGPRs, 4 waves, every group at once.
    float4 a[kFirst];
#pragma unroll
    for (int e = 0; e < kFirst; ++e)
        if ((uint32_t)e < nmax) a[e] = *reinterpret_cast<const float4*>(lv + lslot(seg0, e, ntile));
#pragma unroll
    for (int e = 0; e < kFirst; ++e) {
        const float x[4] = {a[e].x, a[e].y, a[e].z, a[e].w};
#pragma unroll
        for (int q = 0; q < kCountSegs; ++q) c[q] += (uint32_t)e < n[q] && n[q] <= (uint32_t)kCap && fabsf(x[q]) >= tc;
    }
    // longer lists, 8 entries in flight at a time: at 1B a list holds ~7 entries at the
    // list threshold, so most threads have one of their four lists past 8, and a loop of
    // one dependent load per entry made this count phase ~37 us of k_count_emit's ~110
    // (tools/ce_prof.py)
    for (uint32_t e0 = kFirst; e0 < nmax; e0 += kFirst) {
        float4 b[kFirst];
#pragma unroll
        for (int e = 0; e < kFirst; ++e)
            if (e0 + e < nmax) b[e] = *reinterpret_cast<const float4*>(lv + lslot(seg0, e0 + e, ntile));
#pragma unroll
        for (int e = 0; e < kFirst; ++e) {
            if (e0 + e >= nmax) break;
            const float x[4] = {b[e].x, b[e].y, b[e].z, b[e].w};
#pragma unroll
            for (int q = 0; q < kCountSegs; ++q)
                c[q] += e0 + e < n[q] && n[q] <= (uint32_t)kCap && fabsf(x[q]) >= tc;
        }
    }
#pragma unroll
    for (int q = 0; q < kCountSegs; ++q)
        if (ls0 + q < d.nseg && n[q] > (uint32_t)kCap) spill[atomicAdd(&nspill, 1)] = kCountSegs * tid + q;
    __syncthreads();
    for (int i = wave; i < nspill; i += kBlock / kWave) {   // spilled segments: a wave re-reads each
        const int j = spill[i];
        const uint32_t cs = wave_count_segment(vec, d.n, lg * kGroupSegs + j, tc);
        if (lane == 0) spill_cnt[j] = cs;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kCountSegs; ++q)
        if (ls0 + q < d.nseg && n[q] > (uint32_t)kCap) c[q] = spill_cnt[kCountSegs * tid + q];
    CE_STAMP(1);
    const uint32_t mine = c[0] + c[1] + c[2] + c[3];
    uint64_t total;
    const uint32_t tbase = (uint32_t)block_exclusive_scan((uint64_t)mine, lds16, &total);
    uint32_t off[kCountSegs];
    off[0] = tbase;
#pragma unroll
    for (int q = 1; q < kCountSegs; ++q) off[q] = off[q - 1] + c[q - 1];
#pragma unroll
    for (int q = 0; q < kCountSegs; ++q)
        if (ls0 + q < d.nseg) {
            w.seg_cnt[seg0 + q] = c[q];
            w.seg_off[seg0 + q] = off[q];
            if (n[q] > (uint32_t)kCap) spill_cnt[kCountSegs * tid + q] = off[q];   // now its offset
        }
    // the group's offset: decoupled look-back by wave 0, 64 predecessors per poll (one
    // load each, in flight together: a walk of one load at a time paid ~1 us per group)
    if (wave == 0) {
        unsigned long long* lb = w.grp_lb + d.grp0;
        if (lane == 0) {
            if (total) atomicAdd(&w.grp_cnt[d.grp0 + lg], (unsigned long long)total);
            __hip_atomic_store(&lb[lg], (lg == 0 ? kLbPre : kLbAgg) | total, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        unsigned long long prefix = 0;
        bool ok = true;
        int64_t j = lg - 1;   // the window's closest predecessor
        int spin = 0;
        while (j >= 0) {
            const int64_t jj = j - lane;
            // before group 0: an inclusive prefix of 0
            const unsigned long long v =
                jj >= 0 ? __hip_atomic_load(&lb[jj], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbPre;
            const uint64_t pre = __ballot((v & kLbPre) != 0), unready = __ballot(v == 0);
            const int first = pre ? __builtin_ctzll(pre) : kWave;   // the closest inclusive prefix
            const uint64_t need = first >= kWave - 1 ? ~0ull : ((2ull << first) - 1);
            if (unready & need) {   // a group in the window has not published yet: poll again
                if (++spin > kLbSpin) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            prefix += wave_sum(lane <= first ? (v & kLbVal) : 0ull);
            if (first < kWave) break;
            j -= kWave;
        }
        if (lane == 0) {
            if (lg > 0 && ok)
                __hip_atomic_store(&lb[lg], kLbPre | (prefix + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!ok) atomicExch(&st->ce_fail, 1);   // no emit from this group: k_emit will run
            prefix_s = ok ? prefix : ~0ull;
        }
    }
    __syncthreads();
    CE_STAMP(2);
    const unsigned long long P = prefix_s;
    const long long limit = d.k;
    // Payload writes one entry per lane in slot order: a group whose entries fit stages
    // them in LDS and copies them out coalesced (written where they fall, a lane per four
    // lists, they were 4- and 8-B stores to 64 lines per instruction: 81 -> 71 us at 1B).
    const bool emit = P != ~0ull && (long long)P < limit;
    const bool staged = emit && nspill == 0 && total <= (uint64_t)kCeStage;
    if (emit) {
        // the entries >= t_cur at positions P + off + rank < k
        for (uint32_t e0 = 0; e0 < nmax; e0 += kFirst) {
            if ((long long)(P + off[0]) >= limit) break;
            uint2 ob[kFirst];
            float4 vb[kFirst];
#pragma unroll
            for (int e = 0; e < kFirst; ++e)
                if (e0 + e < nmax) {
                    ob[e] = *reinterpret_cast<const uint2*>(lo + lslot(seg0, e0 + e, ntile));
                    vb[e] = *reinterpret_cast<const float4*>(lv + lslot(seg0, e0 + e, ntile));
                }
#pragma unroll
            for (int e = 0; e < kFirst; ++e) {
                if (e0 + e >= nmax) break;
                const float x[4] = {vb[e].x, vb[e].y, vb[e].z, vb[e].w};
                const uint32_t oo[4] = {ob[e].x & 0xFFFFu, ob[e].x >> 16, ob[e].y & 0xFFFFu, ob[e].y >> 16};
#pragma unroll
                for (int q = 0; q < kCountSegs; ++q)
                    if (e0 + e < n[q] && n[q] <= (uint32_t)kCap && fabsf(x[q]) >= tc) {
                        const uint32_t r = off[q];   // in-group slot
                        if (staged) {
                            stage_v[r] = x[q];
                            stage_i[r] = (uint32_t)(kCountSegs * tid + q) * kSeg + oo[q];
                        } else if ((long long)(P + r) < limit) {
                            emit_one(o, d, (long long)(P + r), (ls0 + q) * kSeg + oo[q], x[q], false);
                        }
                        off[q] = r + 1;
                    }
            }
        }
    }
    if (emit && !staged)
        for (int i = wave; i < nspill; i += kBlock / kWave) {   // spilled segments: a wave re-reads each
            const int j = spill[i];
            emit_reread_firstk(vec, d, lg * kGroupSegs + j, (long long)(P + spill_cnt[j]), limit, 0, tc, o, false);
        }
    CE_STAMP(3);
    if (staged) {
        __syncthreads();
        const long long m = std::min<long long>((long long)total, limit - (long long)P);
        const int64_t gbase = lg * kGroupSegs * (int64_t)kSeg;   // the group's first element
        for (long long i = tid; i < m; i += kBlock) {
            store_value(o.values, (long long)P + i, stage_v[i], o.vdtype);
            store_index(o.indices, (long long)P + i, d.idx_base + gbase + stage_i[i], o.idtype);
        }
    }
    CE_STAMP(4);
    // the tensor's last workgroup takes the adaptation step
    if (last_block_arrival8(st->tk8, (uint32_t)lg, (uint32_t)(w.bt[BT_CNT][1] - w.bt[BT_CNT][0])))
        decide_tensor(w, p, 0, 1);
    CE_STAMP(5);
}

__global__ void __launch_bounds__(kBlock)
k_count_emit(const float* __restrict__ vec_flat, SelWS w, SelCfg p, EmitOut o) {
    count_emit_body(vec_flat, w, p, o);
}

// k_count_emit beside the full select pass in ONE launch (one tensor; see k_count_pass):
// the first ncnt workgroups count (and emit) from the lists, the rest re-list over vec
// when the lists do not serve — one of the two does work. The merged kernel keeps the
// select pass's occupancy (its VGPRs bound both; k_count_emit's LDS does not).
template <bool ALIGNED>
__global__ void __launch_bounds__(kBlock)
k_count_emit_pass(const float* __restrict__ vec_flat, SelWS w, SelCfg p, EmitOut o, int which, int ncnt) {
    if ((int)blockIdx.x < ncnt)
        count_emit_body(vec_flat, w, p, o);
    else
        select_pass_body<ALIGNED>(vec_flat, w, which, p, (int64_t)blockIdx.x - ncnt);
}

// Result records; the payload's total count; and every tensor's next speculative
// list threshold, margin x t_cur x growth. One workgroup (any size): k_sel_finish, or
// the last workgroup of k_nth_select.
struct FinishArgs {
    int64_t* count_out;
    dgc_select_info* info;
    float margin;
    int32_t defer, mask_mmt;
    int32_t on;   // k_nth_select: its last workgroup runs the finish (no k_sel_finish launch)
    // Host-mapped (pinned) word of the engine, may be null: a call whose resample replay
    // broke (DGC_K5_BROKEN) stores its status there — a plain system-scope store, only
    // then — so an engine that never synchronises sees it on its next step, for free.
    int32_t* sink;
    uint32_t force;   // DGC_K5_FORCE_BROKEN (tests): status bits added to every resampled tensor
    // may be null: set to DGC_ORDER_ASCENDING when every emitted index of the call is in
    // ascending order (no tensor took the exact replay's topk order), else 0 — the
    // packed payload's header word 1, read by the W = 1 scatter (whole-granule stores)
    int64_t* order_out;
    float margin_max;   // the adaptive list margin's ceiling (kSpecMarginMax; DGC_SPEC_MARGIN_MAX for A/B runs)
};

__device__ __forceinline__ void sel_finish_body(const SelWS& w, const FinishArgs& f) {
    int64_t* count_out = f.count_out;
    dgc_select_info* info = f.info;
    const float margin = f.margin;
    const int defer = f.defer, mask_mmt = f.mask_mmt;
    __shared__ unsigned long long total;
    __shared__ uint32_t broken, topk_order;
    if (threadIdx.x == 0) {
        total = 0;
        broken = 0;
        topk_order = 0;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < w.T; t += blockDim.x) {
        // every load first, by value (a store through st, info or spec could alias a
        // later load: interleaved they were one dependent memory round trip each, 6.5 us
        // for ResNet-50's 54 tensors), then the stores
        // (the fields it uses, one by one: a copy of the whole state indexed by the epoch
        // gave the finish a 1.2 KB/lane scratch frame — k_nth_select 13 -> 22 us at 1B)
        SelState* st = w.st + t;
        struct {
            float t0, t_cur;
            int32_t branch, recounts, overflow, full_passes, list_spills, epoch, tie_rule, win_keys;
            long long n_cur, limit;
        } s;
        s.t0 = st->t0;
        s.t_cur = st->t_cur;
        s.branch = st->branch;
        s.recounts = st->recounts;
        s.overflow = st->overflow;
        s.full_passes = st->full_passes;
        s.list_spills = st->list_spills;
        s.epoch = st->epoch;
        s.tie_rule = st->tie_rule;
        s.win_keys = st->win_keys;
        s.n_cur = st->n_cur;
        s.limit = st->limit;
        const uint32_t wc = st->win_cnt[s.epoch & 1];   // this call's window, taken or not
        const int64_t k = w.td[t].k;
        const bool tail = w.td[t].tail;
        const uint32_t status = w.nthg[t].status;
        float* spec = w.spec ? w.spec + kSpecWords * t : nullptr;
        const float used = spec ? spec[0] : __builtin_huge_valf();
        const float prev = spec ? spec[1] : __builtin_huge_valf();
        const uint32_t k5 = status | (s.branch == DGC_BRANCH_RESAMPLE ? f.force : 0u);
        if (k5 & DGC_K5_BROKEN) atomicOr(&broken, k5);
        // the exact replays (K5, K5b) emit torch.topk's order; every other branch ascends
        if (s.branch == DGC_BRANCH_RESAMPLE && s.tie_rule == DGC_TIES_EXACT) atomicOr(&topk_order, 1u);
        const long long cnt = s.branch == DGC_BRANCH_RESAMPLE ? (long long)k : s.limit;   // final_count
        atomicAdd(&total, (unsigned long long)cnt);
        st->epoch = s.epoch + 1;
        // what the next K1 must zero (first-k branches of a deferring engine only)
        st->def_mode = (defer && s.branch != DGC_BRANCH_RESAMPLE && !tail && cnt > 0) ? 1 : 0;
        st->def_t = s.t_cur;
        st->def_limit = s.limit;
        st->def_mask_mmt = mask_mmt;
        if (info) {
            dgc_select_info& r = info[t];
            r.count = cnt;
            r.candidates = s.n_cur;
            r.threshold0 = s.t0;
            r.threshold = s.t_cur;
            r.branch = s.branch;
            r.recounts = s.recounts;
            r.overflow_segments = s.full_passes ? s.overflow : s.list_spills;
            r.full_passes = s.full_passes;
            r.tie_rule = s.tie_rule;
            r.window_keys = s.win_keys;
            r.k5_status = (int32_t)k5;
            r.list_threshold = used;   // (this call's; spec[0] is updated below)
        }
        if (spec) {
            // spec[0]: next call's list threshold = m x t x growth, growth = 2 - spec[1] / t
            //   (linear extrapolation from the previous final threshold spec[1]) clamped to
            //   [1, 1.5]; spec[1] := t. The ratio t / spec[1] overshoots while the growth
            //   decelerates (the accumulating velocity's threshold grows ~linearly). The
            //   margin m adapts: after a call whose threshold landed at or above its list
            //   threshold (a hit), m = 1.05 x that call's list/final ratio, within [margin,
            //   spec[4]] — the lists shrink towards the selection while the threshold moves
            //   predictably (at 1B on the bench's dynamics 4 % of the elements at 0.8 vs
            //   0.7 % at 0.95; ceiling 0.985: flat-1B's step 0.204 -> 0.179 ms past K1, same
            //   box); a miss (the threshold fell below it: a full select pass ran) resets m
            //   to margin and lowers the ceiling spec[4]. A prediction from the SAMPLED threshold series, with
            //   the lower of the last two final/sampled ratios (lists that hold a lowered
            //   threshold's candidates), was measured and dropped: on ResNet-50 its longer
            //   lists cost the list counts and the lowering 23 + 14 + 25 us where these take
            //   14 + 5 + 5, and the full passes stayed (same box, 0.372 vs 0.337 ms/step).
            const float tc = s.t_cur;
            const bool finite = tc == tc && tc > 0.f && tc < __builtin_huge_valf();
            const float gr = fminf(fmaxf(2.f - prev / tc, 1.f), 1.5f);   // first call: 2 - inf -> 1
            // the ceiling learns how closely t follows its prediction: it climbs while the
            // lists hold t (a hit) and steps down after a miss — a threshold that jitters
            // keeps its lists wider, a steady one (the bench's) narrows them to ~1.5 %
            const float c0 = spec[4] < __builtin_huge_valf() ? spec[4] : fmaxf(margin, kSpecCeil0);
            const bool tried = used < __builtin_huge_valf() && tc > 0.f;
            const bool hit = tried && tc >= used;
            const float mcap = !tried ? c0
                                : hit ? fminf(c0 + kSpecCeilUp, fmaxf(margin, f.margin_max))
                                      : fmaxf(c0 - kSpecCeilDown, margin);
            float m = margin;
            if (hit) m = fminf(fmaxf(1.05f * (used / tc), margin), mcap);
            spec[4] = mcap;
            spec[0] = finite ? tc * m * gr : __builtin_huge_valf();
            spec[1] = finite ? tc : __builtin_huge_valf();
            // spec[2]: next call's sample-window threshold = mw x t0 x growth0, growth0 =
            //   2 - spec[3] / t0 clamped to [1, 1.5] (the sampled threshold's own linear
            //   extrapolation), spec[3] := t0. The window must hold >= ks samples and, for
            //   the one-workgroup select (rs_window_wg), <= kWinMax: mw = 0.97 after a window
            //   of that size, 0.985 after a larger one, 0.9 after one that missed (fewer than
            //   ks samples above it: this call's threshold came from the passes over every
            //   sample). The list threshold's margin (~0.95) put 8 ks samples in the window
            //   at 1B, past one workgroup's registers.
            const float t0 = s.t0;
            const bool f0 = t0 == t0 && t0 > 0.f && t0 < __builtin_huge_valf();
            const float g0 = fminf(fmaxf(2.f - spec[3] / t0, 1.f), 1.5f);
            const float mw = wc > (uint32_t)kWinMax ? 0.985f : (s.win_keys > 0 ? 0.97f : 0.9f);
            spec[2] = f0 ? t0 * mw * g0 : __builtin_huge_valf();
            spec[3] = f0 ? t0 : __builtin_huge_valf();
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && count_out) *count_out = (int64_t)total;
    if (threadIdx.x == 0 && f.order_out) *f.order_out = topk_order ? 0 : (int64_t)DGC_ORDER_ASCENDING;
    if (threadIdx.x == 0 && broken && f.sink)
        __hip_atomic_store(f.sink, (int32_t)broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_sel_finish(SelWS w, FinishArgs f) { sel_finish_body(w, f); }

// K5 emit: output slot q <- candidate queue[q] (the topk's order), with values,
// wire casts and the masking of DGCSGDMemory.update.
__global__ void __launch_bounds__(kBlock) k_emit_queue(const float* __restrict__ vec_flat, SelWS w, EmitOut o) {
    const int t = task(w, BT_QUEUE, blockIdx.x);
    const SelState* st = w.st + t;
    if (!(st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 1)) return;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    __shared__ long long obase_s;
    if (threadIdx.x < kWave) {
        const long long b = out_base(w, t);
        if (threadIdx.x == 0) obase_s = b;
    }
    __syncthreads();
    const int64_t q = ((int64_t)blockIdx.x - w.bt[BT_QUEUE][t]) * kQueuePerBlock + threadIdx.x;
    if (q >= d.k) return;
    const uint32_t j = (uint32_t)w.queue[d.cand_off + q];
    emit_one(o, d, obase_s + q, w.cand_idx[d.cand_off + j], w.cand_val[d.cand_off + j]);
}

// K5b: torch's CPU topk on its partial_sort path (k * 64 <= candidates, i.e. a sampled
// threshold >= 64x too low), replayed EXACTLY for every k and N (dgc/compression.py:
// 134-137): std::partial_sort(queue, queue + k, queue + n, greater) over the
// candidates in index order = make_heap of the first k, then every later candidate
// whose key beats the heap's top replaces it (pop_heap), then sort_heap; queue[0..k)
// is the output in that order. Equal keys are indistinguishable to the heap's
// comparisons, so which boundary ties survive and the order of equal keys come from
// its exact layout — the replay runs the same operations on the same layout.
//
//   entries   (|x| key (31 bits) << 33) | element index (33 bits) for N < 2^33; above, the
//             low 33 bits hold a SLOT in [0, k) and the tensor's cand_idx region maps slot ->
//             element index: the heap holds k entries at any time, and an entry that
//             replaces the root takes the root's slot (its key alone is compared, so the
//             replay is the same)
//   layout    node i in LDS for i < kHeapTop (levels 0..13), else in the tensor's K5
//             queue region (>= k entries: cand_cap = min(64k - 1, N) >= k)
//   fill      the workgroup streams vec in index order, block-scans the candidates
//             (|x| >= t_cur) and writes the first k to nodes 0..k-1
//   make_heap level by level, one thread per parent (parents of one level own
//             disjoint subtrees, so this is std::__make_heap's descending order)
//   select    per 2048-element chunk, the candidates that beat the root are compacted
//             in order; wave 0 re-checks each against the live root and replaces it:
//             the min-child path to a leaf is found 5 levels per load (62 lanes load
//             the hole's subtree, the path is resolved with readlanes), then
//             std::__push_heap's stop on the (monotone) path is one ballot, and the
//             shifted nodes are written in parallel
//   sort_heap k - 1 pops by wave 0, the same replacement on a shrinking heap
//   emit      payload slot p <- node p: values, wire casts, DGCSGDMemory.update's masking
//
// Sequential by nature (~k ln(n/k) replacements + k pops); reached only when the
// sampled threshold came out >= 64x too low, never by the benchmarked workloads.
constexpr int kHeapTop = 16383;                  // nodes in LDS (levels 0..13)
constexpr int kHeapChunk = kNthThreads * 4;      // vec elements per step: one float4 per thread
constexpr int kHeapSub = 5;                      // levels of the path resolved per load
constexpr int kHeapKeyShift = 33;
constexpr uint64_t kHeapIdxMask = (1ull << kHeapKeyShift) - 1;
constexpr size_t kHeapSmemBytes = (size_t)(kHeapTop + 1 + kHeapChunk) * 8;   // nodes + hot list
constexpr size_t kK5SmemBytes = kHeapSmemBytes > kNthSmemBytes ? kHeapSmemBytes : kNthSmemBytes;

__device__ __forceinline__ uint32_t hkey(uint64_t e) { return (uint32_t)(e >> kHeapKeyShift); }

struct HeapNodes {
    DGC_LDS uint64_t* l;   // nodes [0, kHeapTop)
    DGC_GLB uint64_t* g;   // nodes >= kHeapTop (indexed by node)
    __device__ __forceinline__ uint64_t ld(int64_t i) const { return i < kHeapTop ? l[i] : g[i]; }
    __device__ __forceinline__ void st(int64_t i, uint64_t v) const {
        if (i < kHeapTop)
            l[i] = v;
        else
            g[i] = v;
    }
};

// std::__adjust_heap + std::__push_heap on nodes [0, len) from `hole` with value v,
// comp = key greater (the root holds the smallest key). One thread (make_heap).
__device__ void heap_adjust1(const HeapNodes& h, int64_t hole, int64_t len, uint64_t v) {
    const int64_t top = hole;
    int64_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        const uint64_t r = h.ld(child), l = h.ld(child - 1);
        uint64_t c = r;
        if (hkey(r) > hkey(l)) {
            child--;
            c = l;
        }
        h.st(hole, c);
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        h.st(hole, h.ld(child - 1));
        hole = child - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top) {
        const uint64_t pv = h.ld(parent);
        if (!(hkey(pv) > hkey(v))) break;
        h.st(hole, pv);
        hole = parent;
        parent = (hole - 1) / 2;
    }
    h.st(hole, v);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// std::__adjust_heap(first, 0, len, v) — the root replaced by v — by ONE wave (all 64
// lanes, uniform arguments). Returns the new root. The min-child path from the root:
// lanes 2^d - 2 .. 2^(d+1) - 3 hold the hole's descendants at depth d = 1..5, loaded
// at once; the choice at each level (right child unless the left key is smaller;
// a lone left child at the end) is resolved from them with readlanes. Along the path
// the keys never decrease (heap order), so push_heap's climb stops at J = the first
// path node whose key exceeds v's: nodes p_0..p_(J-2) take the values of p_1..p_(J-1),
// p_(J-1) takes v, the rest keep theirs — written by lanes 0..J-1 at once.
__device__ uint64_t heap_replace_root(const HeapNodes& h, int64_t len, uint64_t v) {
    const int lane = threadIdx.x & 63;
    uint64_t pidx = 0, pval = 0;   // lane j-1: path node p_j and its value a_j
    int m = 0;                     // path length
    int64_t hole = 0;
    bool more = len > 1;
    while (more) {
        // this lane's descendant of `hole`: depth dl (1..5), offset ol
        const int dl = 31 - __clz(lane + 2);               // lane + 2 in [2^dl, 2^(dl+1))
        const int64_t ol = (int64_t)(lane + 2) - (1ll << dl);
        const int64_t node = ((hole + 1) << dl) - 1 + ol;
        uint64_t val = 0;
        if (lane < 62 && node < len) val = h.ld(node);
        int64_t off = 0;   // the hole's offset among the subtree nodes of its depth
        for (int d = 1; d <= kHeapSub; ++d) {
            const int base = (1 << d) - 2;
            int64_t child;
            uint64_t cval;
            if (hole < (len - 1) / 2) {   // two children
                const uint64_t l = readlane64(val, base + (int)(2 * off));
                const uint64_t r = readlane64(val, base + (int)(2 * off) + 1);
                if (hkey(r) > hkey(l)) {
                    child = 2 * hole + 1;
                    cval = l;
                    off = 2 * off;
                } else {
                    child = 2 * hole + 2;
                    cval = r;
                    off = 2 * off + 1;
                }
            } else if ((len & 1) == 0 && hole == (len - 2) / 2) {   // a lone left child, then stop
                child = 2 * hole + 1;
                cval = readlane64(val, base + (int)(2 * off));
                off = 2 * off;
                more = false;
            } else {
                more = false;
                break;
            }
            if (lane == m) {
                pidx = (uint64_t)child;
                pval = cval;
            }
            ++m;
            hole = child;
            if (!more) break;
        }
    }
    // J - 1 = the first lane (path index) whose value's key exceeds v's; m if none
    const uint64_t above = __ballot(lane < m && hkey(pval) > hkey(v));
    const int jm1 = above ? __builtin_ctzll(above) : m;
    const uint64_t up = (uint64_t)__shfl_up((long long)pidx, 1);
    const int64_t parent = lane == 0 ? 0 : (int64_t)up;   // p_(lane) for lane >= 1, p_0 = root
    if (lane < jm1)
        h.st(parent, pval);   // p_(lane) <- a_(lane+1)
    else if (lane == jm1)
        h.st(parent, v);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the next replacement reads these
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return jm1 == 0 ? v : readlane64(pval, 0);
}

// Chunk loads: 4 consecutive elements of vec per thread, kHeapAhead chunks (16 KB) in
// flight per batch, the next batch issued before the current one is processed — the
// workgroup streams vec at a CU's load rate instead of one round trip per chunk.
constexpr int kHeapAhead = 8;

__device__ __forceinline__ void heap_load(const float* vec, int64_t n, int64_t c0, bool al, float (&x)[4]) {
    const int64_t e0 = c0 + 4 * (int64_t)threadIdx.x;
    if (al && e0 + 3 < n) {
        const float4 v = *reinterpret_cast<const float4*>(vec + e0);
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = e0 + j < n ? vec[e0 + j] : 0.f;
    }
}

// Candidate bits of a thread's 4 elements at chunk c0 (|x| >= tc; NaN never is).
__device__ __forceinline__ uint32_t heap_cands(int64_t n, int64_t c0, float tc, const float (&x)[4]) {
    const int64_t e0 = c0 + 4 * (int64_t)threadIdx.x;
    uint32_t cm = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) cm |= (uint32_t)(e0 + j < n && fabsf(x[j]) >= tc) << j;
    return cm;
}

// Streams the chunks from c_begin in index order, kHeapAhead at a time with the next
// batch in flight; f(c0, x) returns false to stop (uniformly). Returns the chunk it
// stopped at (n rounded up to a chunk when it ran to the end).
template <class F>
__device__ __forceinline__ int64_t heap_stream(const float* vec, int64_t n, int64_t c_begin, bool al, F&& f) {
    constexpr int64_t kBatch = (int64_t)kHeapAhead * kHeapChunk;
    float xa[kHeapAhead][4], xb[kHeapAhead][4];
#pragma unroll
    for (int u = 0; u < kHeapAhead; ++u) heap_load(vec, n, c_begin + u * kHeapChunk, al, xa[u]);
    for (int64_t b0 = c_begin; b0 < n; b0 += kBatch) {
#pragma unroll
        for (int u = 0; u < kHeapAhead; ++u) heap_load(vec, n, b0 + kBatch + u * kHeapChunk, al, xb[u]);
#pragma unroll
        for (int u = 0; u < kHeapAhead; ++u) {
            const int64_t c0 = b0 + u * kHeapChunk;
            if (c0 >= n) return c0;
            if (!f(c0, xa[u])) return c0;
        }
#pragma unroll
        for (int u = 0; u < kHeapAhead; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) xa[u][j] = xb[u][j];
    }
    return n;
}

__device__ __forceinline__ void heap_select_wg(const float* __restrict__ vec_flat, const SelWS& w, const EmitOut& o, int t,
                               uint64_t* smem) {
    const SelState* st = w.st + t;
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const float* vec = vec_flat + d.off;
    const float tc = st->t_cur;
    const int64_t k = d.k, n = d.n;
    const bool al = aligned16(vec);
    const HeapNodes h{lds(smem), glb(w.queue + d.cand_off)};
    // wide (N >= 2^33): node payloads are slots, side[slot] the element index
    const bool wide = n >= ((int64_t)1 << kHeapKeyShift);
    DGC_GLB int64_t* side = glb(w.cand_idx + d.cand_off);
    uint64_t* hot = smem + kHeapTop + 1;
    __shared__ uint64_t lds16[16];
    __shared__ uint64_t root_sh;
    __shared__ long long obase_s;
    const int tid = threadIdx.x;
    // ---- fill: the first k candidates, in index order, become nodes 0..k-1
    int64_t filled = 0, skip = 0;   // skip: candidates of the last fill chunk that went into the heap
    const int64_t c_fill = heap_stream(vec, n, 0, al, [&](int64_t c0, const float (&x)[4]) -> bool {
        const uint32_t cm = heap_cands(n, c0, tc, x);
        uint64_t total;
        uint64_t r = block_exclusive_scan((uint64_t)__popc(cm), lds16, &total);
        const int64_t e0 = c0 + 4 * (int64_t)tid;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if ((cm >> j) & 1u) {
                const int64_t g = filled + (int64_t)r++;
                if (g < k) {
                    h.st(g, ((uint64_t)abs_key(x[j]) << kHeapKeyShift) | (uint64_t)(wide ? g : e0 + j));
                    if (wide) side[g] = e0 + j;
                }
            }
        }
        if (filled + (int64_t)total >= k) {
            skip = k - filled;
            filled = k;
            return false;
        }
        filled += (int64_t)total;
        return true;
    });
    __syncthreads();
    // ---- make_heap, level by level (deepest parents first)
    if (k >= 2) {
        const int64_t last_parent = (k - 2) / 2;
        const int top_level = 63 - __clzll((unsigned long long)(last_parent + 1));
        for (int lv = top_level; lv >= 0; --lv) {
            const int64_t p0 = (1ll << lv) - 1;
            const int64_t p1 = std::min<int64_t>((2ll << lv) - 2, last_parent);
            for (int64_t p = p0 + tid; p <= p1; p += kNthThreads) heap_adjust1(h, p, k, h.ld(p));
            __syncthreads();
        }
    }
    // ---- heap select over the candidates after the first k, from the chunk the fill ended in
    if (tid == 0) root_sh = h.ld(0);
    __syncthreads();
    heap_stream(vec, n, c_fill, al, [&](int64_t c0, const float (&x)[4]) -> bool {
        const uint32_t cm = heap_cands(n, c0, tc, x);
        const uint32_t rk = hkey(root_sh);
        uint32_t hm = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) hm |= (uint32_t)(((cm >> j) & 1u) && abs_key(x[j]) > rk) << j;
        if (skip > 0) {   // the chunk where the fill ended: its first `skip` candidates are in the heap
            uint64_t tot;
            uint64_t r = block_exclusive_scan((uint64_t)__popc(cm), lds16, &tot);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((cm >> j) & 1u) {
                    if ((int64_t)r < skip) hm &= ~(1u << j);
                    ++r;
                }
            skip = 0;
        }
        if (!__syncthreads_or(hm != 0)) return true;
        uint64_t htot;
        const uint64_t hb = block_exclusive_scan((uint64_t)__popc(hm), lds16, &htot);
        uint64_t q = hb;
        // hot entries carry the element's offset in this chunk (< kHeapChunk)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((hm >> j) & 1u) hot[q++] = ((uint64_t)abs_key(x[j]) << kHeapKeyShift) | (uint64_t)(4 * tid + j);
        __syncthreads();
        if (tid < kWave) {   // wave 0: comp(candidate, top) is "strictly greater"
            uint64_t root = root_sh;
            for (uint64_t i = 0; i < htot; ++i) {
                const uint64_t hv = hot[i];
                if (hkey(hv) > hkey(root)) {
                    const int64_t e = c0 + (int64_t)(hv & kHeapIdxMask);
                    const uint64_t slot = root & kHeapIdxMask;   // the popped root's slot is recycled
                    if (wide && tid == 0) side[slot] = e;
                    const uint64_t v = (hv & ~kHeapIdxMask) | (uint64_t)(wide ? (int64_t)slot : e);
                    root = heap_replace_root(h, k, v);
                }
            }
            if (tid == 0) root_sh = root;
        }
        __syncthreads();
        return true;
    });
    // ---- sort_heap: k - 1 pops by wave 0
    if (tid < kWave) {
        for (int64_t last = k - 1; last >= 1; --last) {
            const uint64_t v = h.ld(last);
            const uint64_t root = h.ld(0);
            if (tid == 0) h.st(last, root);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            (void)heap_replace_root(h, last, v);
        }
    }
    __syncthreads();
    // ---- emit: payload slot p <- node p
    if (tid < kWave) {
        const long long b = out_base(w, t);
        if (tid == 0) obase_s = b;
    }
    __syncthreads();
    for (int64_t p = tid; p < k; p += kNthThreads) {
        const int64_t lo = (int64_t)(h.ld(p) & kHeapIdxMask);
        const int64_t li = wide ? side[lo] : lo;
        emit_one(o, d, obase_s + p, li, vec[li]);
    }
}

// K5 / K5b, one workgroup per tensor: the reference's resample topk replayed on the
// gathered candidates (introselect.hpp: nth_element), or — partial_sort path — heap
// select + sort_heap over vec, which also emits. They share one LDS area.
static_assert(kK5SmemBytes <= 160 * 1024 - 1024, "K5 / K5b LDS");
// ---------------------------------------------------------------- K5s: a resample's set
// For an engine (resample_order = 1) a resampled tensor's payload need not list torch's
// topk order: the exchange's decompress (index_put_ of distinct indices) and
// DGCSGDMemory.update depend on the SET of the top-k (dgc/compression.py:134-137,
// 179-194; dgc/memory.py:72-77). When the k-th largest candidate key is not tied
// across the k boundary (#keys >= kth == k) every top-k is that set, whatever order
// and tie rule produced it, so it is emitted in index order and the exact replay (K5)
// skips the tensor (rs_nth = 3). Tied, the replay runs as always. The k-th largest is
// found by a radix select over key - key(t_cur) (every candidate is >= t_cur) in three
// 11-bit passes over the open range up to 0x7FFFFFFF; the emit carries the wire casts
// and the masking of the K5 emit.
//
// Over G co-resident workgroups of ONE launch (the tensor's BT_SET workgroups: kSetG,
// up to kSetGBig for a capacity past kSetG x kSetCoopMin — VGG-16-BN's fc6, where four
// sliced launches k_bigset_* ran as no-ops every step before; one for a capacity up to
// kSetCoopMin, and none for a tensor that cannot resample — a fixed 16 per tensor took
// ~10 us to dispatch): a set of more than kSetCoopMin candidates is cut into G contiguous
// stretches of rounds, each workgroup's keys in its registers; the radix passes'
// histograms and the per-stretch counts go through device atomics with a barrier
// between the phases (pass 1 | pass 2 | pass 3 | counts), and each
// workgroup emits its stretch's selected entries at the count of the stretches before
// it plus their order inside it — the index order, as one workgroup emits it. A set of
// up to kSetRegC x 1024 candidates takes the same code on one workgroup, with no
// barrier. The G workgroups start with a residency consensus (as K5's global phase):
// should they not all be resident within kSetArriveTicks, the tensor is left to the
// exact replay (k_nth_select), exact either way; so is a barrier that times out (not
// expected after the consensus), and a tie across the k boundary as before.
// (ResNet-50's 72k-candidate resample: one workgroup walked its keys six times, 24 of
// 72 rounds from L2 — 59 us of the step.)
constexpr uint64_t kSetArriveTicks = 200000;   // 2 ms of the 100 MHz wall clock
static_assert(kSetCoopMin == (int64_t)kSetRegC * kScanThreads, "K5s: one workgroup holds kSetCoopMin keys");

__device__ __forceinline__ bool setg_consensus(SetG* g, uint32_t G) {
    __shared__ uint32_t verdict;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t a = __hip_atomic_fetch_add(&g->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a + 1 == G) {
            atomicCAS(&g->decide, (uint32_t)kNthGUndecided, (uint32_t)kNthGGo);
        } else {
            const uint64_t t0 = wall_clock64();
            while (__hip_atomic_load(&g->decide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kNthGUndecided) {
                if (wall_clock64() - t0 > kSetArriveTicks) {
                    atomicCAS(&g->decide, (uint32_t)kNthGUndecided, (uint32_t)kNthGAbort);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        verdict = __hip_atomic_load(&g->decide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return verdict == kNthGGo;
}

// Barrier among the G workgroups: everything they exchange is device atomics, read back
// with agent-scope atomic loads (last_block_arrival's "atomics both sides"), so draining
// this workgroup's atomics (vmcnt(0)) before the arrival is the only ordering needed.
__device__ __forceinline__ void setg_barrier(SetG* g, uint32_t G, uint32_t* status) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t gen = __hip_atomic_load(&g->bar_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t a = __hip_atomic_fetch_add(&g->bar_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a == G - 1) {
            __hip_atomic_store(&g->bar_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&g->bar_gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            bool passed = false;
            for (uint32_t spin = 0; spin < (1u << 24); ++spin) {
                if (__hip_atomic_load(&g->bar_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) {
                    passed = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!passed) {   // the replay takes the tensor (exact); recorded for the caller
                __hip_atomic_store(&g->broken, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicOr(status, (uint32_t)DGC_K5_SET_BROKEN);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// (OVF: a stretch longer than the registers hold — a set above ~2M candidates; the
// common case compiles without the L2 rounds)
template <bool OVF>
__device__ __forceinline__ void resample_set_body(const float* __restrict__ vec_flat, const SelWS& w, const EmitOut& o,
                                                  int t, uint32_t b, uint32_t G, int per, int rounds,
                                                  SelState* st, const TDesc& d) {
    const int64_t n64 = st->n_cur;
    SetG* g = w.setg + t;
    if (G > 1 && !setg_consensus(g, G)) {   // not all resident: the replay (recorded for the caller)
        if (b == 0 && threadIdx.x == 0) atomicOr(&w.nthg[t].status, (uint32_t)DGC_K5_SET_FALLBACK);
        return;
    }
    SET_STAMP(0);
    const int n = (int)n64;
    const uint32_t k = (uint32_t)d.k;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int kWaves = kScanThreads / kWave;
    __shared__ uint32_t h[kSetBins1];
    __shared__ uint32_t lds32[16];
    __shared__ uint32_t rbase[(OVF ? kSetRoundsMax : kSetRegC) * kWaves];
    __shared__ uint32_t sel_above, sel_cnt, s_base, s_stop;
    __shared__ int sel_bin;
    __shared__ long long obase_s;
    // this workgroup's stretch of rounds; queue entry i = tid + r * 1024 (coalesced)
    const int r0 = (int)b * per, r1 = min(r0 + per, rounds);
    const DGC_GLB uint32_t* qk = glb(w.cand_key + d.cand_off);
    auto valid = [&](int r) { return r0 + r < r1 && tid + (r0 + r) * kScanThreads < n; };
    uint32_t key[kSetRegC];
#pragma unroll
    for (int r = 0; r < kSetRegC; ++r) key[r] = valid(r) ? qk[tid + (r0 + r) * kScanThreads] : 0u;
    // every round of the stretch: the registers, then (a big set only) the rest from L2
    auto walk = [&](auto&& f) {
#pragma unroll
        for (int r = 0; r < kSetRegC; ++r) f(r, key[r], valid(r));
        if (OVF)
            for (int r = kSetRegC; r < per; ++r) {
                const bool v = valid(r);
                f(r, v ? qk[tid + (r0 + r) * kScanThreads] : 0u, v);
            }
    };
    // the key range: every candidate has |x| >= t_cur (the gather's test), so key(t_cur)
    // bounds it from below, and the two passes cover kSetSpan bits above it (4 octaves):
    // the first pass's top bin also takes every key past that span, and should the k-th
    // largest fall there the replay takes the tensor (exact either way). Two passes of
    // 4096 and 8192 bins, not three of 2048: each pass of a cooperative set is a merge
    // and a barrier (~5 us over 16 workgroups). A min/max phase over the keys cost a
    // barrier too (2.2 us in one workgroup, 5.5 us over 16); an open range up to
    // 0x7FFFFFFF piled the first pass into a few bins (LDS atomics on the same words:
    // +8 us in one workgroup, tools/k5s_prof.py).
    const uint32_t mn = abs_key(st->t_cur);
    for (int q = tid; q < kSetBins1; q += kScanThreads) h[q] = 0;
    __syncthreads();
    SET_STAMP(1);
    static_assert(kSetBins0 == 4 * kScanThreads && kSetBins1 == 8 * kScanThreads, "pick_bin_small<4 | 8>");
    int passes = 0;   // (whose merged histograms this workgroup re-zeroes its share of)
    uint32_t prefix = 0, k_rem = k;
    uint32_t kth = mn, eq = (uint32_t)n;
    bool ok = true;
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t nb = pass == 0 ? (uint32_t)kSetBins0 : (uint32_t)kSetBins1;
        walk([&](int, uint32_t kk, bool v) {
            const uint32_t x = kk - mn;
            if (!v) return;
            if (pass == 0) atomicAdd(&h[min(x >> kSetLo0, nb - 1u)], 1u);
            else if ((x >> kSetLo0) == prefix) atomicAdd(&h[x & (nb - 1u)], 1u);
        });
        __syncthreads();
        if (G > 1) {   // every workgroup picks the same bin from the same merged histogram
            uint32_t* gh = pass == 0 ? g->hist0 : g->hist1;
            for (int q = tid; q < (int)nb; q += kScanThreads)
                if (h[q]) __hip_atomic_fetch_add(&gh[q], h[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            setg_barrier(g, G, &w.nthg[t].status);
            for (int q = tid; q < (int)nb; q += kScanThreads)
                h[q] = __hip_atomic_load(&gh[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
        }
        if (tid == 0) sel_bin = -1;
        __syncthreads();
        int bin;
        uint32_t above;
        const bool hit = pass == 0 ? pick_bin_small<4>(h, k_rem, lds32, &bin, &above)
                                   : pick_bin_small<8>(h, k_rem, lds32, &bin, &above);
        if (hit) {
            sel_bin = bin;
            sel_above = above;
            sel_cnt = h[bin];
        }
        __syncthreads();
        const int sb = sel_bin;
        const uint32_t a = sel_above, c = sel_cnt;
        __syncthreads();   // every thread has read sel_*
        for (int q = tid; q < (int)nb; q += kScanThreads) h[q] = 0;
        __syncthreads();   // zeroed before the next pass's adds (a wave ahead lost counts to a late zero)
        passes = pass + 1;
        if (sb < 0 || (pass == 0 && sb == kSetBins0 - 1)) {   // (sb < 0 cannot happen: k < n keys)
            ok = false;   // the k-th largest is 4 octaves or more above t_cur: the replay takes it
            break;
        }
        k_rem -= a;
        if (pass == 0) {
            prefix = (uint32_t)sb;
        } else {
            kth = mn + ((prefix << kSetLo0) | (uint32_t)sb);
            eq = c;
        }
    }
    __syncthreads();
    // tied across the boundary (more keys == kth than the k - #(> kth) still needed):
    // only torch's exact order of operations knows which ones — the replay
    if (eq != k_rem) ok = false;
    SET_STAMP(2);
    // order-preserving compaction: (round, wave) ballot counts, one workgroup scan, the
    // stretches before this one (their counts through the last barrier)
    walk([&](int r, uint32_t kk, bool v) {
        const uint32_t c = ok ? (uint32_t)__popcll(__ballot(v && kk >= kth)) : 0u;
        if (lane == 0) rbase[r * kWaves + wv] = c;
    });
    __syncthreads();
    {
        const uint32_t c = tid < per * kWaves ? rbase[tid] : 0u;
        uint32_t total;
        const uint32_t run = block_exclusive_scan32(c, lds32, &total);
        if (tid < per * kWaves) rbase[tid] = run;
        if (tid == 0) {
            s_base = 0;
            s_stop = ok ? 0u : 1u;
            if (G > 1) __hip_atomic_store(&g->cnt[b], total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    static_assert(kSetRoundsMax * kWaves <= kScanThreads, "one compaction count per thread");
    if (G > 1) {
        setg_barrier(g, G, &w.nthg[t].status);
        if (tid == 0) {
            uint32_t base = 0;
            for (uint32_t i = 0; i < b; ++i)
                base += __hip_atomic_load(&g->cnt[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_base = base;
            if (__hip_atomic_load(&g->broken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) s_stop = 1;
        }
        // every workgroup has read the histograms: re-zero this one's share of those used
        for (int p = 0; p < passes; ++p) {
            const int nb = p == 0 ? kSetBins0 : kSetBins1, share = (nb + (int)G - 1) / (int)G;
            uint32_t* gh = p == 0 ? g->hist0 : g->hist1;
            const int qlo = (int)b * share, qhi = min(qlo + share, nb);
            for (int q = qlo + tid; q < qhi; q += kScanThreads) gh[q] = 0;
        }
    }
    if (wv == 0) {
        const long long ob = out_base(w, t);
        if (lane == 0) obase_s = ob;
    }
    __syncthreads();
    if (s_stop) return;   // uniform: a tie or a broken barrier — the replay takes the tensor
    SET_STAMP(3);
    const long long ob = obase_s + (long long)s_base;
    const int64_t* cand = w.cand_idx + d.cand_off;
    const float* cval = w.cand_val + d.cand_off;
    // the register rounds 8 at a time, every selected candidate's index and value loaded
    // before the first store (the stores may alias the loads, so a round-by-round walk
    // waited out a load round trip per round: 12 us for 16k candidates in one workgroup)
    constexpr int kEmitRounds = 8;
    static_assert(kSetRegC % kEmitRounds == 0, "emit batches");
#pragma unroll
    for (int r0b = 0; r0b < kSetRegC; r0b += kEmitRounds) {
        int64_t ci[kEmitRounds];
        float cv[kEmitRounds];
        bool sl[kEmitRounds];
#pragma unroll
        for (int j = 0; j < kEmitRounds; ++j) {
            const int r = r0b + j;
            sl[j] = valid(r) && key[r] >= kth;
            const int i = tid + (r0 + r) * kScanThreads;
            ci[j] = sl[j] ? cand[i] : 0;
            cv[j] = sl[j] ? cval[i] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < kEmitRounds; ++j) {
            const uint64_t mm = __ballot(sl[j]);
            if (sl[j]) emit_one(o, d, ob + rbase[(r0b + j) * kWaves + wv] + mbcnt64(mm, 0u), ci[j], cv[j]);
        }
    }
    if (OVF)
        for (int r = kSetRegC; r < per; ++r) {
            const int i = tid + (r0 + r) * kScanThreads;
            const bool sel = valid(r) && qk[i] >= kth;
            const uint64_t mm = __ballot(sel);
            if (sel) emit_one(o, d, ob + rbase[r * kWaves + wv] + mbcnt64(mm, 0u), cand[i], cval[i]);
        }
    if (b == 0 && tid == 0) {
        st->rs_nth = 3;   // K5's replay and emit skip the tensor
        st->tie_rule = DGC_TIES_SET;
    }
    SET_STAMP(4);
}

// One workgroup of k_resample_set (bx: its index in the BT_SET grid). wait: k_emit_set,
// whose emit workgroups gather the candidates in the same launch — the set's workgroups
// first wait until all of the tensor's emit workgroups have counted themselves (bounded:
// past kSetArriveTicks the tensor is left to the exact replay, recorded as a fallback).
__device__ __forceinline__ void resample_set_block(const float* __restrict__ vec_flat, const SelWS& w,
                                                   const EmitOut& o, int bx, int64_t one_max, uint32_t gmin,
                                                   bool wait) {
    const int t = task(w, BT_SET, bx);
    const uint32_t b = (uint32_t)bx - (uint32_t)w.bt[BT_SET][t];
    SelState* st = w.st + t;
    if (st->branch != DGC_BRANCH_RESAMPLE || st->rs_nth != 1) return;   // uniform per workgroup
    const TDesc d = w.td[t];   // by value: stores below cannot alias it
    const uint32_t Gt = (uint32_t)(w.bt[BT_SET][t + 1] - w.bt[BT_SET][t]);   // this tensor's workgroups
    const int64_t n64 = st->n_cur;
    if (d.k < 1 || n64 <= d.k) return;
    // this set's workgroups: one up to kSetCoopMin candidates, else kSetG, and for a big
    // tensor as many as keep its stretches in registers (up to Gt); each stretch's rounds
    // past the registers are read from L2 on every walk, up to kSetRoundsMax per stretch
    const int rounds = (int)((n64 + kScanThreads - 1) / kScanThreads);
    uint32_t G = 1;
    if (n64 > one_max && Gt > 1) {   // (then Gt >= gmin: n64 <= cand_cap)
        const uint32_t want = (uint32_t)((rounds + kSetRegC - 1) / kSetRegC);
        G = want > gmin ? (want < Gt ? want : Gt) : gmin;
        G = G < Gt ? G : Gt;
    }
    const int per = (rounds + (int)G - 1) / (int)G;
    if (per > kSetRoundsMax || b >= G) return;   // (past kSetRoundsMax: the replay)
    if (wait) {
        __shared__ int gathered;
        if (threadIdx.x == 0) {
            const uint32_t want = (uint32_t)(w.bt[BT_GRP][t + 1] - w.bt[BT_GRP][t]);
            const uint64_t t0 = wall_clock64();
            bool ok = true;
            while (__hip_atomic_load(&w.setg[t].gathered, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                if (wall_clock64() - t0 > kSetArriveTicks) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (!ok) atomicOr(&w.nthg[t].status, (uint32_t)DGC_K5_SET_FALLBACK);
            gathered = ok;
        }
        __syncthreads();
        ES_STAMP(1);
        // (a cooperative set's other workgroups then fail the residency consensus: the replay)
        if (!gathered) return;
    }
    if (per > kSetRegC)
        resample_set_body<true>(vec_flat, w, o, t, b, G, per, rounds, st, d);
    else
        resample_set_body<false>(vec_flat, w, o, t, b, G, per, rounds, st, d);
}

__global__ void __launch_bounds__(kScanThreads)
k_resample_set(const float* __restrict__ vec_flat, SelWS w, EmitOut o, int64_t one_max, uint32_t gmin) {
    resample_set_block(vec_flat, w, o, (int)blockIdx.x, one_max, gmin, false);
}

// K5's global-memory phase by G workgroups per tensor (grid G x T, a plain launch sized
// so all of them fit at once; a residency consensus decides whether they run it, see
// introselect.hpp); k_nth_select goes on from the state it leaves. The A/B form
// (DGC_NTH_SEPARATE=1): by default k_nth_select runs the phase on its own extra
// workgroups (grid T x G), one launch fewer.
__global__ void __launch_bounds__(kNthThreads) k_nth_global(SelWS w, uint32_t G, int64_t min_run,
                                                            uint32_t G_expected) {
    __shared__ uint8_t mk[kNthGMk];
    const int t = blockIdx.y;
    const SelState* st = w.st + t;
    if (st->branch != DGC_BRANCH_RESAMPLE || st->rs_nth != 1) return;
    const TDesc d = w.td[t];
    uint32_t* gl = w.gpos + d.gpos_off;
    uint32_t* gr = gl + d.cand_cap / 2 + 1;
    nth_global_multi(w.queue + d.cand_off, st->n_cur, d.k - 1, gl, gr, w.nthg + t, blockIdx.x, G, min_run,
                     G_expected, lds(mk));
}

// Grid T x G: workgroup (t, 0) replays tensor t; with G > 1 and `global_here` the
// tensor's G workgroups (t, 0..G-1) first run K5's global phase (nth_global_multi, its
// stopper bytes in the replay's LDS area, which is free until the phase ends), and
// workgroups (t, b > 0) leave after it. from_global: G > 1, the phase ran (here or in
// k_nth_global) and the replay goes on from the state it left.
// The last of the T workgroups (t, 0) to finish (f.on) then runs the finish of the whole
// call (T arrivals on one ticket; nothing it writes is read by k_emit_queue).
//
// A global phase that BROKE (a barrier timed out after the consensus voted GO: its
// partitions of the queue are not reliable) is recovered here, in the same call: the
// queue is rebuilt from the gather's candidate keys — entry j = (key_j << 32 | j), as
// the gather wrote it — and the whole nth_element replayed on this workgroup from
// [0, n), exact (k5_status DGC_K5_FALLBACK | DGC_K5_RECOVERED). force_broken (parity
// tests, DGC_K5_FORCE_BROKEN=1): every replayed tensor takes that path, its queue first
// overwritten with garbage.
// queue_here (k > kQueueFold somewhere, and G > 1 workgroups per tensor): the extra
// workgroups (t, 1..G-1) of a replayed tensor wait for its replay (NthG::replayed) and
// write its k entries in the replayed order, a share each — k_emit_queue, a ~5 us
// launch that is a no-op in every step without a replay (flat-1B, VGG-16-BN), is not
// launched. The wait is bounded (~seconds; workgroup (t, 0) never waits on them): past
// it the payload is incomplete and the call reports DGC_K5_BROKEN through the sink.
__global__ void __launch_bounds__(kNthThreads) k_nth_select(const float* __restrict__ vec_flat, SelWS w,
                                                            EmitOut o, int from_global, FinishArgs f,
                                                            int force_broken, int emit_here, int global_here,
                                                            uint32_t G, int64_t min_run, uint32_t G_expected,
                                                            int queue_here, int rebuild_queue) {
    const int t = blockIdx.x;
    const uint32_t b = blockIdx.y;
    const SelState* st = w.st + t;
    __shared__ __align__(16) uint64_t smem[kK5SmemBytes / 8];
    static_assert(kK5SmemBytes >= (size_t)kNthGMk, "the global phase's stopper bytes fit the replay's LDS");
    if (global_here && st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 1) {   // uniform per tensor
        const TDesc d = w.td[t];
        uint32_t* gl = w.gpos + d.gpos_off;
        uint32_t* gr = gl + d.cand_cap / 2 + 1;
        nth_global_multi(w.queue + d.cand_off, st->n_cur, d.k - 1, gl, gr, w.nthg + t, b, G, min_run, G_expected,
                         reinterpret_cast<DGC_LDS uint8_t*>(lds(smem)));
        __syncthreads();   // (smem is the replay's from here)
    }
    if (b > 0) {
        if (queue_here && st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 1) {   // uniform per tensor
            NthG* g = w.nthg + t;
            __shared__ int ready;
            __shared__ long long qbase_s;
            if (threadIdx.x == 0) {
                bool done = false;
                for (uint32_t spin = 0; spin < (1u << 26); ++spin) {
                    if (__hip_atomic_load(&g->replayed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        done = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (!done) {
                    atomicOr(&g->status, (uint32_t)DGC_K5_BROKEN);
                    raise_flag(f.sink, (int32_t)DGC_K5_BROKEN);
                }
                ready = done;
            }
            __syncthreads();
            if (!ready) return;   // uniform
            if (threadIdx.x < kWave) {
                const long long ob = out_base(w, t);
                if (threadIdx.x == 0) qbase_s = ob;
            }
            __syncthreads();
            const TDesc d = w.td[t];
            const int64_t share = ceil_div(d.k, (int64_t)(G - 1));
            const int64_t q0 = (int64_t)(b - 1) * share, q1 = q0 + share < d.k ? q0 + share : d.k;
            for (int64_t q = q0 + threadIdx.x; q < q1; q += kNthThreads) {
                const uint32_t j = (uint32_t)w.queue[d.cand_off + q];
                emit_one(o, d, qbase_s + q, w.cand_idx[d.cand_off + j], w.cand_val[d.cand_off + j]);
            }
        }
        return;
    }
    K5_STAMP(7);
    if (st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 2) {   // uniform per workgroup
        heap_select_wg(vec_flat, w, o, t, smem);
    } else if (st->branch == DGC_BRANCH_RESAMPLE && st->rs_nth == 1) {
        const TDesc d = w.td[t];   // by value: stores below cannot alias it
        DGC_GLB uint32_t* gl = glb(w.gpos + d.gpos_off);
        DGC_GLB uint32_t* gr = gl + d.cand_cap / 2 + 1;
        DGC_LDS uint64_t* lq = lds(smem);
        DGC_LDS uint32_t* llp = reinterpret_cast<DGC_LDS uint32_t*>(lq + kNthLds);
        DGC_LDS uint32_t* lrp = llp + kNthPairLds;
        DGC_LDS uint8_t* lmk = reinterpret_cast<DGC_LDS uint8_t*>(lrp + kNthPairLds);
        NthG* g = w.nthg + t;
        DGC_GLB uint64_t* q = glb(w.queue + d.cand_off);
        const int64_t nc = st->n_cur;
        __shared__ int recover;
        if (threadIdx.x == 0)
            recover = force_broken ||
                      (from_global && (__hip_atomic_load(&g->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                                       (uint32_t)DGC_K5_BROKEN));
        __syncthreads();
        if (recover) {
            // a GO phase's workgroups may still be on their way out of a timed-out barrier
            // (here, not k_nth_global): none touches the queue once it has counted itself
            if (global_here && threadIdx.x == 0 &&
                __hip_atomic_load(&g->decide, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kNthGGo)
                while (__hip_atomic_load(&g->exited, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < G)
                    __builtin_amdgcn_s_sleep(2);
            __syncthreads();
            if (force_broken)
                for (int64_t j = threadIdx.x; j < nc; j += kNthThreads) q[j] = ~(uint64_t)j;
            __syncthreads();
            const DGC_GLB uint32_t* ck = glb(w.cand_key + d.cand_off);
            for (int64_t j = threadIdx.x; j < nc; j += kNthThreads) q[j] = ((uint64_t)ck[j] << 32) | (uint64_t)j;
            __syncthreads();
            if (threadIdx.x == 0)
                g->status = (g->status & ~(uint32_t)DGC_K5_BROKEN) | (uint32_t)(DGC_K5_FALLBACK | DGC_K5_RECOVERED);
        } else if (rebuild_queue) {   // the gather wrote no queue (an index-order engine, no global phase)
            const DGC_GLB uint32_t* ck = glb(w.cand_key + d.cand_off);
            for (int64_t j = threadIdx.x; j < nc; j += kNthThreads) q[j] = ((uint64_t)ck[j] << 32) | (uint64_t)j;
            __syncthreads();
        }
        nth_element_wg(q, nc, d.k - 1, gl, gr, lq, llp, lrp, lmk, from_global && !recover ? g : nullptr);
        if (queue_here) {   // the replayed order is in the queue: the extra workgroups emit it
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                __hip_atomic_store(&g->replayed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (emit_here) {
            // the replayed order out by this workgroup (k <= kQueueFold for every tensor of
            // the call: no k_emit_queue launch); the payload position is known, every
            // tensor's branch and count being final before K5 runs
            __shared__ long long obase_s;
            __syncthreads();
            if (threadIdx.x < kWave) {
                const long long b = out_base(w, t);
                if (threadIdx.x == 0) obase_s = b;
            }
            __syncthreads();
            const long long ob = obase_s;
            for (int64_t q0 = threadIdx.x; q0 < d.k; q0 += kNthThreads) {
                const uint32_t j = (uint32_t)q[q0];
                emit_one(o, d, ob + q0, w.cand_idx[d.cand_off + j], w.cand_val[d.cand_off + j]);
            }
        }
    }
    const bool idle = !(st->branch == DGC_BRANCH_RESAMPLE && (st->rs_nth == 1 || st->rs_nth == 2));
    if (idle) K5_STAMP(0);   // (profiling build: slots 0-2 are free when the replay did not run)
    if (f.on && last_block_arrival(w.fin_ticket, gridDim.x)) {
        if (idle) K5_STAMP(1);
        sel_finish_body(w, f);
        if (idle) K5_STAMP(2);
    }
    K5_STAMP(6);
}

__global__ void k_spec_reset(float* spec, int32_t T) {
    for (int i = threadIdx.x; i < kSpecWords * T; i += blockDim.x) spec[i] = __builtin_huge_valf();
}

// ------------------------------------------------------------------ host driver
// The resample replays pack what they move into 64-bit entries: K5's queue holds
// (key << 32 | candidate position), K5b's heap (key31 << 33 | element index, or a slot
// of the k heap entries with the index beside it from N = 2^33 on). A tensor whose
// candidates do not fit K5's width is refused up front — torch's topk takes any n
// (dgc/compression.py:124-137), and a truncated position would be a wrong payload, not
// an error. (k < 2^32 follows: the candidate capacity min(64k - 1, n) is >= k.)
static int check_replay_width(int64_t n, int64_t k, const char* who) {
    if (nth_cand_cap(n, k) > (int64_t)0xFFFFFFFFLL)
        DGC_FAIL(DGC_ERR_OVERFLOW,
                 "%s: the resample replay addresses at most 2^32 - 1 candidates; numel %lld with num_selects %lld "
                 "can have %lld (use resample=False or a smaller tensor)",
                 who, (long long)n, (long long)k, (long long)nth_cand_cap(n, k));
    return DGC_OK;
}

static int validate_select(const dgc_select_params* p, void* values, void* indices) {
    if (!p) DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null params");
    if (p->numel < 1 || p->num_selects < 1 || p->num_selects > p->numel)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: need 1 <= num_selects <= numel (got %lld, %lld)",
                 (long long)p->num_selects, (long long)p->numel);
    if (p->num_samples < 1 || p->num_samples > p->numel)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: bad num_samples");
    if (p->max_iters < 0) DGC_FAIL(DGC_ERR_INVALID, "dgc_select: max_iters < 0");
    if (p->vdtype != DGC_F32 && p->vdtype != DGC_F16 && p->vdtype != DGC_BF16)
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_select: value dtype");
    if (p->thr_dtype != DGC_F32 && p->thr_dtype != DGC_F16 && p->thr_dtype != DGC_BF16)
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_select: threshold dtype");
    if (p->idtype != DGC_I64 && p->idtype != DGC_I32) DGC_FAIL(DGC_ERR_DTYPE, "dgc_select: index dtype");
    if (p->idtype == DGC_I32 && p->numel > 2147483647LL)
        DGC_FAIL(DGC_ERR_OVERFLOW, "dgc_select: int32 indices cannot address %lld elements",
                 (long long)p->numel);
    if (p->resample) DGC_TRY(check_replay_width(p->numel, p->num_selects, "dgc_select"));
    if (!values || !indices) DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null outputs");
    return DGC_OK;
}

static SelCfg cfg_of(const dgc_select_params& p) {
    return SelCfg{p.upper, p.lower,       p.max_iters,     p.resample,  p.masking,
                  p.vdtype, p.idtype,     p.update_memory, p.thr_dtype, p.resample_order == 1 ? 1 : 0};
}

// The selection of every tensor (its K1 lists kept or not), from k_sel_init to the
// payload: stream-ordered, and in DGC_SYNC_DEVICE mode with no host synchronisation.
// k_emit for many groups (flat buckets), k_emit_wide for few (model gradient sets).
// DGC_EMIT_SHAPE=quarter|wide forces one (the parity tests run both at small sizes).
static bool emit_is_wide(const Layout& L) {
    const char* force = std::getenv("DGC_EMIT_SHAPE");
    return force ? std::strcmp(force, "wide") == 0 : L.ngrp < 256;
}

static int launch_emit(const Layout& L, const float* vec, const SelWS& w, const EmitOut& o, hipStream_t s) {
    if (emit_is_wide(L))
        hipLaunchKernelGGL(k_emit_wide_t<false>, dim3((unsigned)L.grid[BT_GRP]), dim3(kGroupSegs), 0, s, vec, w, o, o,
                           (int64_t)0, 0u, (int32_t)L.grid[BT_GRP]);
    else
        hipLaunchKernelGGL(k_emit, dim3((unsigned)L.grid[BT_GRP]), dim3(kEmitSegs), 0, s, vec, w, o);
    DGC_LAUNCHED();
    return DGC_OK;
}

// Workgroups per tensor for K5's global phase (k_nth_select's extra workgroups, or
// k_nth_global's): half the CUs shared among the T tensors, at most kNthGMax. They wait
// for each other, so all of them must be resident at once: <= CUs / 2 workgroups of 8
// waves (one fits a CU, with k_nth_select's ~150 KB of LDS as with k_nth_global's 33 KB)
// guarantee that with this stream's earlier kernels done. (hipLaunchCooperativeKernel checks the same
// but cost ~29 us per launch on MI355X: more than the phase saves below ~200k candidates.)
// <= 1 runs the one-workgroup global phase inside k_nth_select instead; so does a call
// whose tensors all have candidate capacities <= kNthGMinCand, and so does a tensor
// with <= kNthGMinCand candidates (decided on the device: below ~100k the three
// cross-XCD barriers per step cost as much as the spread saves, tools/run_k5.sh), and
// DGC_K5_GLOBAL=wg (A/B, parity); DGC_K5_GLOBAL=multi skips both gates.
constexpr int64_t kNthGMinCand = 98304;    // launch for capacities above, run for candidate counts above

static uint32_t nth_global_groups(int32_t T, int64_t max_cand) {
    static int per_dev = -1;
    if (per_dev < 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_nth_select),
                                                         kNthThreads, 0) != hipSuccess)
            per_dev = 0;
        else
            per_dev = per_cu >= 1 ? cus / 2 : 0;

    }
    const char* force = std::getenv("DGC_K5_GLOBAL");   // wg | multi (parity tests run both)
    if (force && std::strcmp(force, "wg") == 0) return 0;
    const bool multi = force && (std::strcmp(force, "multi") == 0 || std::strcmp(force, "abort") == 0);
    if (max_cand <= kNthLds || (max_cand <= kNthGMinCand && !multi)) return 0;
    // measured (tools/run_k5.sh): 16 workgroups per tensor for every tensor of a batch
    // from 40k candidates made ResNet-50 0.358 -> 0.373 ms (864 workgroups launched per
    // step, and at 45-57k candidates the spread phase is no faster than one workgroup:
    // 0.141-0.144 ms either way); it pays from ~100k (500k: 0.945 -> 0.371 ms)
    // fewer than 4 per tensor (a batch of many tensors: ResNet-50's 54) spread too little
    // to pay the barriers, and the launch alone is ~5.7 us per step (rocprofv3)
    const int64_t g = T > 0 ? per_dev / T : 0;
    if (g < 4 && !multi) return 0;
    return (uint32_t)std::min<int64_t>(g, kNthGMax);
}

static int select_core(float* vec, float* mmt, const SelCfg& p, const Layout& L, void* values, void* indices,
                       int64_t* count_out, dgc_select_info* info, const SelWS& w, int keep_lists, int sync_mode,
                       float margin, int32_t* sink, int64_t* order_out, hipStream_t s) {
    // keep_lists: a compress call, whose K3 kernels already reset every tensor's state
    // (sel_init_tensor) when they produced its threshold; a pure selection resets here
    if (!keep_lists) {
        hipLaunchKernelGGL(k_sel_init, dim3((unsigned)L.T), dim3(kScanThreads), 0, s, w, 0);
        DGC_LAUNCHED();
    }
    const bool al = aligned16(vec);
    // resample=True with max_iters <= kMaxLower: one multi-threshold pass replaces the lowers
    const bool lower_fast = p.resample && p.max_iters <= kMaxLower;
    EmitOut o{p.update_memory ? vec : nullptr, (p.update_memory && p.masking) ? mmt : nullptr, values, indices,
              p.vdtype, p.idtype, nullptr, nullptr, (int32_t)(p.update_memory == 2)};
    // the first list count of a one-tensor call also writes the first-k payload
    // (k_count_emit) when that emit would not mask and the payload starts at slot 0
    const bool fuse = keep_lists && L.T == 1 && !L.tail_any && sync_mode == DGC_SYNC_DEVICE &&
                      (p.update_memory == 2 || p.update_memory == 0) && !std::getenv("DGC_NO_COUNT_EMIT");
    static const bool pass_split = std::getenv("DGC_PASS_SPLIT") != nullptr;
    static const int pass_super = [] {
        const char* e = std::getenv("DGC_PASS_SUPER");
        const int v = e ? std::atoi(e) : 2;
        return v == 1 || v == 2 ? v : kSuper;
    }();
    const bool merge_ok = lower_fast && sync_mode == DGC_SYNC_DEVICE && !pass_split;
    auto pass = [&](int need, bool likely_lists, bool fused = false) -> int {
        // one count pass at t_cur: lists when t_cur >= t_list, else the full select pass
        // (both gated per tensor on the device); need: 1 = lists, 2 = full, 3 = either
        // each count kernel's last workgroup per tensor takes the adaptation step
        if (need == 3 && fused && merge_ok) {   // both in one launch (k_count_emit_pass)
            const int which = likely_lists ? BT_CAP16 : BT_FULL;
            const unsigned grid = (unsigned)(L.grid[BT_CNT] + L.grid[which]);
            if (al)
                hipLaunchKernelGGL(k_count_emit_pass<true>, dim3(grid), dim3(kBlock), 0, s, vec, w, p, o, which,
                                   (int)L.grid[BT_CNT]);
            else
                hipLaunchKernelGGL(k_count_emit_pass<false>, dim3(grid), dim3(kBlock), 0, s, vec, w, p, o, which,
                                   (int)L.grid[BT_CNT]);
            DGC_LAUNCHED();
            return DGC_OK;
        }
        if (need == 3 && !fused && merge_ok) {   // both in one launch (k_count_pass)
            // a batch's full passes: two segments per wave (DGC_PASS_SUPER=1|4: one or
            // kSuper, A/B). Measured (tools/pass_prof.py, ResNet-50): four per wave keep
            // a working workgroup ~9 us on its list appends after 3 us of loads, one per
            // wave ~3 us but 6289 workgroups enter over 10.7 us (the working ones hold
            // the slots); two: 6 us each, all entered within 3.9 us, the pass ends at 15
            // instead of 18 us — ResNet-50 0.2269 -> 0.2235 ms, VGG-16-BN 0.6275 -> 0.6264
            // (4 alternations; one per wave 0.2310 / 0.6282)
            const int sup = L.T > 1 ? pass_super : kSuper;
            const int which = sup == 1 ? (likely_lists ? BT_CAP4 : BT_K1)
                            : sup == 2 ? (likely_lists ? BT_CAP8 : BT_FULL8) : (likely_lists ? BT_CAP16 : BT_FULL);
            const unsigned grid = (unsigned)(L.grid[BT_CNT] + L.grid[which]);
            if (sup == 1 && al)
                hipLaunchKernelGGL((k_count_pass<true, 1>), dim3(grid), dim3(kBlock), 0, s, vec, w, which, p,
                                   (int)L.grid[BT_CNT]);
            else if (sup == 1)
                hipLaunchKernelGGL((k_count_pass<false, 1>), dim3(grid), dim3(kBlock), 0, s, vec, w, which, p,
                                   (int)L.grid[BT_CNT]);
            else if (sup == 2 && al)
                hipLaunchKernelGGL((k_count_pass<true, 2>), dim3(grid), dim3(kBlock), 0, s, vec, w, which, p,
                                   (int)L.grid[BT_CNT]);
            else if (sup == 2)
                hipLaunchKernelGGL((k_count_pass<false, 2>), dim3(grid), dim3(kBlock), 0, s, vec, w, which, p,
                                   (int)L.grid[BT_CNT]);
            else if (al)
                hipLaunchKernelGGL((k_count_pass<true, kSuper>), dim3(grid), dim3(kBlock), 0, s, vec, w, which, p,
                                   (int)L.grid[BT_CNT]);
            else
                hipLaunchKernelGGL((k_count_pass<false, kSuper>), dim3(grid), dim3(kBlock), 0, s, vec, w, which, p,
                                   (int)L.grid[BT_CNT]);
            DGC_LAUNCHED();
            return DGC_OK;
        }
        if (need & 1) {
            if (fused)
                hipLaunchKernelGGL(k_count_emit, dim3((unsigned)L.grid[BT_CNT]), dim3(kBlock), 0, s, vec, w, p, o);
            else
                hipLaunchKernelGGL(k_count_lists, dim3((unsigned)L.grid[BT_CNT]), dim3(kBlock), 0, s, vec, w, p);
            DGC_LAUNCHED();
        }
        if (need & 2) {
            const int which = likely_lists ? BT_CAP16 : BT_FULL;
            const unsigned grid = (unsigned)L.grid[which];
            if (al)
                hipLaunchKernelGGL(k_select_pass<true>, dim3(grid), dim3(kBlock), 0, s, vec, w, which, p);
            else
                hipLaunchKernelGGL(k_select_pass<false>, dim3(grid), dim3(kBlock), 0, s, vec, w, which, p);
            DGC_LAUNCHED();
        }
        return DGC_OK;
    };
    // the lowering from the K1 lists first, then over vec if they do not reach: for one
    // tensor (the per-tensor path; the flat bucket chains its lowering, k_chain_one). A
    // batch goes to vec at once: on per-step gradients a lowered threshold (0.8 t0) sits
    // below the lists almost always, and the list launch cost ResNet-50 6 us, VGG-16-BN 4
    // (same box, 3 alternations); DGC_LOWER_LISTS=0/1 overrides
    static const int lower_lists_env = [] {
        const char* e = std::getenv("DGC_LOWER_LISTS");
        return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
    }();
    const bool lower_lists = lower_lists_env >= 0 ? lower_lists_env == 1 : L.T == 1;
    static const int lower_segs = std::getenv("DGC_LOWER_SEGS") && std::atoi(std::getenv("DGC_LOWER_SEGS")) == 2 ? 2 : 1;
    auto lower = [&]() -> int {
        if (lower_lists) {
            hipLaunchKernelGGL(k_lower_lists, dim3((unsigned)L.grid[BT_SEG]), dim3(kBlock), 0, s, vec, w, p);
            DGC_LAUNCHED();
        }
        // (DGC_LOWER_SEGS=2: two segments per wave over half the workgroups — A/B)
        const bool two = lower_segs == 2;
        const unsigned grid = (unsigned)L.grid[two ? BT_CAP8 : BT_CAP4];
        if (two && al)
            hipLaunchKernelGGL((k_lower_counts<true, 2>), dim3(grid), dim3(kBlock), 0, s, vec, w, p);
        else if (two)
            hipLaunchKernelGGL((k_lower_counts<false, 2>), dim3(grid), dim3(kBlock), 0, s, vec, w, p);
        else if (al)
            hipLaunchKernelGGL((k_lower_counts<true, 1>), dim3(grid), dim3(kBlock), 0, s, vec, w, p);
        else
            hipLaunchKernelGGL((k_lower_counts<false, 1>), dim3(grid), dim3(kBlock), 0, s, vec, w, p);
        DGC_LAUNCHED();
        return DGC_OK;
    };
    // DGC_K5_FORCE_BROKEN=1 (parity tests only): every replayed tensor takes the recovery
    // of a broken global phase (k_nth_select), without a barrier actually timing out
    const int force = std::getenv("DGC_K5_FORCE_BROKEN") ? 1 : 0;
    static const float margin_max = [] {
        const char* e = std::getenv("DGC_SPEC_MARGIN_MAX");
        return e ? std::strtof(e, nullptr) : kSpecMarginMax;
    }();
    const FinishArgs fin{count_out, info, margin, (int32_t)(p.update_memory == 2), (int32_t)(p.masking != 0), 0,
                         sink, 0u, order_out, margin_max};
    bool finished = false;   // the payload count and records are written
    // one tensor, device decisions, the lowering shortcut: the lowering and the count at
    // the lowered threshold in one launch (k_chain_one); DGC_NO_CHAIN=1 (A/B runs)
    // launches them one by one
    static const bool no_chain = std::getenv("DGC_NO_CHAIN") != nullptr;
    static const bool chain_batch = std::getenv("DGC_CHAIN_BATCH") != nullptr;   // (A/B: the batches too)
    const bool chained = (L.T == 1 || chain_batch) && keep_lists && sync_mode == DGC_SYNC_DEVICE && lower_fast &&
                         !no_chain;
    EmitOut g = o;   // the K5 gather (+ every other tensor's payload)
    g.queue = w.queue;
    g.cand = w.cand_idx;
    g.cval = w.cand_val;
    g.ckey = w.cand_key;
    // A/B switches (defaults measured): the one-workgroup limit of a K5s set,
    // the replay's own emit for small k, the merged count pass, the lowering from lists
    static const int64_t set_one_max = [] {
        const char* e = std::getenv("DGC_SET_ONE");
        return e ? std::max<int64_t>(std::atoll(e), 1) : kSetOneMax;
    }();
    static const bool queue_launch = std::getenv("DGC_QUEUE_LAUNCH") != nullptr;
    const bool emit_here = !queue_launch && L.max_k <= kQueueFold;
    auto resample_exact = [&]() -> int {
        // nth_element path: gather candidates, replay the introselect, emit in its order.
        // The gather launch also emits every other tensor's payload (the final emit).
        const uint32_t G = nth_global_groups(L.T, L.max_cand);
        // An index-order engine whose replay runs on one workgroup (no global phase): the
        // gather writes no queue — the sets read the keys, and the rare tied set that
        // falls to the replay has k_nth_select rebuild its queue from them (one of the
        // gather's four stores per candidate; DGC_GATHER_QUEUE=1 writes it, A/B)
        static const bool gather_queue = std::getenv("DGC_GATHER_QUEUE") != nullptr;
        const bool no_queue = p.set_order && G <= 1 && !gather_queue;
        g.no_queue = no_queue ? 1 : 0;
        // K5s: an untied resample set in index order (the rest: the replay); with the
        // wide emit, in its launch (k_emit_set; DGC_SET_SEPARATE=1: two launches, A/B)
        static const bool set_separate = std::getenv("DGC_SET_SEPARATE") != nullptr;
        const bool sets = p.set_order && L.grid[BT_SET] > 0;
        if (sets && !set_separate && emit_is_wide(L)) {
            hipLaunchKernelGGL(k_emit_wide_t<true>, dim3((unsigned)(L.grid[BT_GRP] + L.grid[BT_SET])),
                               dim3(kGroupSegs), 0, s, vec, w, g, o, set_one_max, set_gmin(), (int32_t)L.grid[BT_GRP]);
            DGC_LAUNCHED();
        } else {
            DGC_TRY(launch_emit(L, vec, w, g, s));
            if (sets) {
                hipLaunchKernelGGL(k_resample_set, dim3((unsigned)L.grid[BT_SET]), dim3(kScanThreads), 0, s, vec, w,
                                   o, set_one_max, set_gmin());
                DGC_LAUNCHED();
            }
        }
        // DGC_K5_GLOBAL=multi: every range over several workgroups (parity); =abort: the
        // kernel expects one workgroup more than launched, so the residency consensus
        // times out and the one-workgroup replay takes over (the fallback's parity test)
        const char* gforce = std::getenv("DGC_K5_GLOBAL");
        const bool multi = gforce && (std::strcmp(gforce, "multi") == 0 || std::strcmp(gforce, "abort") == 0);
        const bool abort = gforce && std::strcmp(gforce, "abort") == 0;
        const int64_t min_run = multi ? 0 : kNthGMinCand;
        const uint32_t G_expected = abort ? G + 1 : G;
        static const bool nth_separate = std::getenv("DGC_NTH_SEPARATE") != nullptr;
        const bool global_here = G > 1 && !nth_separate;
        if (G > 1 && !global_here) {
            hipLaunchKernelGGL(k_nth_global, dim3(G, (unsigned)L.T), dim3(kNthThreads), 0, s, w, G, min_run,
                               G_expected);
            DGC_LAUNCHED();
        }
        FinishArgs f = fin;
        f.on = 1;   // k_nth_select's last workgroup finishes the call
        // (DGC_QUEUE_LAUNCH=1 above: always k_emit_queue, A/B)
        const bool queue_here = !emit_here && global_here && !queue_launch;
        hipLaunchKernelGGL(k_nth_select, dim3((unsigned)L.T, global_here ? G : 1u), dim3(kNthThreads), 0, s, vec, w,
                           o, G > 1 ? 1 : 0, f, force, emit_here ? 1 : 0, global_here ? 1 : 0, G, min_run, G_expected,
                           queue_here ? 1 : 0, no_queue ? 1 : 0);
        DGC_LAUNCHED();
        finished = true;
        if (!emit_here && !queue_here) {
            hipLaunchKernelGGL(k_emit_queue, dim3((unsigned)L.grid[BT_QUEUE]), dim3(kBlock), 0, s, vec, w, o);
            DGC_LAUNCHED();
        }
        return DGC_OK;
    };
    DGC_TRY(keep_lists ? pass(3, true, fuse) : pass(2, false));
    bool emitted = false;   // the payload of every non-K5 tensor is written
    if (sync_mode == DGC_SYNC_HOST) {
        // read the decisions back and launch only what they need
        std::vector<SelState> hs(L.T);
        for (;;) {
            DGC_HIP(hipMemcpyAsync(hs.data(), w.st, sizeof(SelState) * L.T, hipMemcpyDeviceToHost, s));
            DGC_HIP(hipStreamSynchronize(s));
            bool all_done = true, any_lower = false, any_full = false, any_list = false;
            for (const SelState& h : hs) {
                if (h.done) continue;
                all_done = false;
                if (h.lower_pending)
                    any_lower = true;
                else if (h.t_cur >= h.t_list)
                    any_list = true;
                else
                    any_full = true;
            }
            if (all_done) break;
            if (any_lower) {
                DGC_TRY(lower());   // picks t_cur on the device: either pass may follow
                DGC_TRY(pass(3, false));
            } else {
                DGC_TRY(pass((any_list ? 1 : 0) | (any_full ? 2 : 0), false));
            }
        }
        bool any_resample = false;
        for (const SelState& h : hs) any_resample |= h.branch == DGC_BRANCH_RESAMPLE;
        if (any_resample) {   // k_nth_select serves both paths (K5, K5b)
            DGC_TRY(resample_exact());
            emitted = true;
        }
    } else if (L.adapt_any) {
        // every kernel below early-exits on a device flag when it is not needed
        if (chained) {   // lower() and pass(3)'s count in one launch, then its full pass
            const unsigned grid = (unsigned)std::min<int64_t>(
                kCapBlocks, std::max({L.grid[BT_SEG], L.grid[BT_CAP4], L.grid[BT_CNT]}));
            if (al)
                hipLaunchKernelGGL(k_chain_one<true>, dim3(grid), dim3(kBlock), 0, s, vec, w, p);
            else
                hipLaunchKernelGGL(k_chain_one<false>, dim3(grid), dim3(kBlock), 0, s, vec, w, p);
            DGC_LAUNCHED();
            DGC_TRY(pass(2, true));
        } else if (lower_fast) {
            DGC_TRY(lower());
            DGC_TRY(pass(3, true));
        } else {
            for (int i = 0; i < p.max_iters; ++i) DGC_TRY(pass(3, true));
        }
        if (p.resample) {
            DGC_TRY(resample_exact());
            emitted = true;
        }
    }
    if (!emitted) DGC_TRY(launch_emit(L, vec, w, o, s));
    if (!finished) {
        hipLaunchKernelGGL(k_sel_finish, dim3(1), dim3(256), 0, s, w, fin);
        DGC_LAUNCHED();
    }
    return DGC_OK;
}

// ------------------------------------------------------------------ one-tensor plumbing
// Layout + table of one unpadded tensor. samples: reserve the strided-sample buffer.
static void one_layout(const dgc_select_params& p, int64_t stride, int64_t ks, bool samples, Layout& L,
                       OneTable& ot) {
    TensorIn in{p.numel, 0, p.num_selects, p.num_samples, ks, stride, p.upper_count, p.lower_count, samples};
    std::vector<TDesc> td;
    std::vector<int32_t> bt[BT_COUNT];
    std::vector<int32_t> small;
    build_layout(&in, 1, false, L, td, bt, small);
    ot.d = td[0];
    for (int which = 0; which < BT_COUNT; ++which) {
        ot.bt[which][0] = bt[which][0];
        ot.bt[which][1] = bt[which][1];
    }
    ot.start = 0;
}

static size_t one_ws_bytes(int64_t numel, int64_t k, int64_t num_samples, bool samples) {
    dgc_select_params p{};
    p.numel = numel;
    p.num_selects = k;
    p.num_samples = num_samples;
    Layout L;
    OneTable ot{};
    one_layout(p, 2, 1, samples, L, ot);
    size_t b = 0;
    carve_select(nullptr, L, &b);
    return b;
}

static size_t select_ws_bytes(int64_t numel, int64_t k) { return one_ws_bytes(numel, k, numel, false); }

int select(float* vec, float* mmt, const float* thr0, const dgc_select_params* p, void* values, void* indices,
           int64_t* count_out, dgc_select_info* info, void* ws, size_t ws_bytes, int sync_mode, hipStream_t s) {
    DGC_TRY(validate_select(p, values, indices));
    if (!vec || !thr0 || (p->update_memory && p->masking && !mmt))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_select: null vec/thr0/mmt");
    Layout L;
    OneTable ot{};
    one_layout(*p, 1, 1, false, L, ot);
    size_t need = 0;
    carve_select(nullptr, L, &need);
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_select: workspace needs %zu bytes, 256-B aligned", need);
    SelWS w = carve_select(ws, L);
    w.spec = nullptr;
    w.thr = const_cast<float*>(thr0);
    hipLaunchKernelGGL(k_put_one, dim3(1), dim3(64), 0, s, w, ot);
    DGC_LAUNCHED();
    return select_core(vec, mmt, cfg_of(*p), L, values, indices, count_out, info, w, 0, sync_mode, 1.f,
                       p->status_sink, p->order_out, s);
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
    RSState* st = reinterpret_cast<RSState*>(ws);
    hipLaunchKernelGGL(k_rs_init, dim3(1), dim3(kBlock), 0, s, st, (uint64_t)k);
    DGC_LAUNCHED();
    return radix_select_passes(DenseKeys{x, n, st, out}, grid_for(n, kBlock * 16, 512), s);
}

// K3 of every tensor of the call: the small ones in one workgroup each, the rest in
// three multi-block passes.
static int thresholds(const SelWS& w, const Layout& L, const float* vec, hipStream_t s, int64_t ks1 = 0) {
    if (L.nsmall + L.nwins) {
        // DGC_NO_WIN_HIST=1 (A/B runs): the window's keys only, not K1's histogram of them
        static const int use_hist = std::getenv("DGC_NO_WIN_HIST") ? 0 : 1;
        hipLaunchKernelGGL(k_rs_small_multi, dim3((unsigned)(L.nsmall + L.nwins)), dim3(kScanThreads), 0, s, w, vec,
                           ks1, L.nsmall, use_hist);
        DGC_LAUNCHED();
    }
    if (L.grid[BT_SAMP] > 0) {
        if (L.nplain) {   // (a windowed task's reset is k_rs_small_multi's)
            hipLaunchKernelGGL(k_rs_reset_samples, dim3((unsigned)L.T), dim3(kBlock), 0, s, w, ks1);
            DGC_LAUNCHED();
        }
        // DGC_NO_RS_CHAIN=1 (A/B runs): the three passes as three launches
        static const bool no_chain = std::getenv("DGC_NO_RS_CHAIN") != nullptr;
        if (no_chain) {
            DGC_TRY(radix_select_passes(SampleKeys{w, vec}, (int)L.grid[BT_SAMP], s));
        } else {
            const int grid = (int)L.grid[BT_SAMP];
            hipLaunchKernelGGL(k_rs_passes<SampleKeys>, dim3((unsigned)std::min(grid, 1024)), dim3(kBlock), 0, s,
                               SampleKeys{w, vec}, grid, (int)L.T);
            DGC_LAUNCHED();
        }
    }
    return DGC_OK;
}

// ------------------------------------------------------------------ fused compress (one tensor)
int compensate(const float* grad, float* mmt, float* vec, float* out, int64_t n, float momentum,
               bool nesterov, bool accumulate, float* samples, int64_t s_start, int64_t s_stride,
               int64_t s_count, hipStream_t st);
int sample_strided_launch(const float* vec, int64_t start, int64_t stride, int64_t count, float* out,
                          hipStream_t s);

static int compress_check(const dgc_select_params* p, void* values, void* indices, int64_t s_start,
                          int64_t s_stride, int64_t top_k_samples, bool need_outputs) {
    if (need_outputs) DGC_TRY(validate_select(p, values, indices));
    else if (!p) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: null params");
    else if (p->resample) DGC_TRY(check_replay_width(p->numel, p->num_selects, "dgc_compress"));
    const bool sampled = p->numel != p->num_samples;
    if (sampled && (s_stride < 2 || s_start < 0 || s_start >= s_stride))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: sample_start must be in [0, stride)");
    const int64_t cnt = sampled ? ceil_div(p->numel - s_start, s_stride) : p->numel;
    if (need_outputs && (top_k_samples < 1 || top_k_samples > cnt))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: top_k_samples %lld outside [1, %lld]", (long long)top_k_samples,
                 (long long)cnt);
    return DGC_OK;
}

static int one_ws(const dgc_select_params* p, int64_t s_start, int64_t s_stride, int64_t ks, float* spec,
                  void* ws, size_t ws_bytes, Layout& L, SelWS& w, OneTable& ot) {
    one_layout(*p, s_stride, ks, true, L, ot);
    ot.start = p->numel != p->num_samples ? s_start : 0;
    size_t need = 0;
    carve_select(nullptr, L, &need);
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_compress: workspace needs %zu bytes, 256-B aligned", need);
    w = carve_select(ws, L);
    w.spec = spec;   // the caller's per-tensor float[kSpecWords] (null: no speculative lists)
    return DGC_OK;
}

// K1 (+ fused strided sample + speculative candidate lists at spec[0]).
int compress_begin(const float* grad, float* mmt, float* vec, float momentum, bool nesterov, int64_t s_start,
                   int64_t s_stride, const dgc_select_params* p, float* spec, void* ws, size_t ws_bytes,
                   hipStream_t s) {
    DGC_TRY(compress_check(p, nullptr, nullptr, s_start, s_stride, 1, false));
    if (!grad || !mmt || !vec) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: null grad/mmt/vec");
    Layout L;
    SelWS w;
    OneTable ot{};
    DGC_TRY(one_ws(p, s_start, s_stride, 1, spec, ws, ws_bytes, L, w, ot));
    const int64_t n = p->numel;
    const bool sampled = n != p->num_samples;
    const int64_t cnt = sampled ? ceil_div(n - s_start, s_stride) : 0;
    const bool list_path = aligned16(grad) && aligned16(mmt) && aligned16(vec) &&
                           (!sampled || (s_stride >= 4 && s_stride < (1LL << 30)));
    if (!list_path) {
        hipLaunchKernelGGL(k_put_one, dim3(1), dim3(64), 0, s, w, ot);
        DGC_LAUNCHED();
        DGC_TRY(mask_flush(vec, mmt, L, w, s));   // a deferring finish left its masking to K1
        DGC_TRY(compensate(grad, mmt, vec, nullptr, n, momentum, nesterov, true, sampled ? w.samples : nullptr,
                           s_start, s_stride, cnt, s));
        hipLaunchKernelGGL(k_no_lists, dim3(1), dim3(64), 0, s, w);
        DGC_LAUNCHED();
        return DGC_OK;
    }
    if (L.grid[BT_K1] > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: n too large");
    if (L.grid[BT_K1] > 0) {
        StartChunk one{};   // the start (and the tables, ot) in the arguments: no k_put_one
        one.count = 1;
        one.start[0] = ot.start;
        if (nesterov)
            hipLaunchKernelGGL((k_compensate_list<true, true>), dim3((unsigned)L.grid[BT_K1]), dim3(kBlock), 0, s,
                               grad, mmt, vec, momentum, w, one, (int)write_through(n), ot);
        else
            hipLaunchKernelGGL((k_compensate_list<false, true>), dim3((unsigned)L.grid[BT_K1]), dim3(kBlock), 0, s,
                               grad, mmt, vec, momentum, w, one, (int)write_through(n), ot);
        DGC_LAUNCHED();
    } else {
        hipLaunchKernelGGL(k_put_one, dim3(1), dim3(64), 0, s, w, ot);
        DGC_LAUNCHED();
    }
    if (n & 3) {   // scalar tail (< 4 elements) incl. its samples; its segment is marked spilled
        const int64_t done = (n / 4) * 4;
        DGC_TRY(compensate(grad + done, mmt + done, vec + done, nullptr, n - done, momentum, nesterov, true, nullptr,
                           0, 1, 0, s));
        if (sampled) {
            // samples in the tail: start + q*stride >= done
            const int64_t q_first = done >= s_start ? ceil_div(done - s_start, s_stride) : 0;
            const int64_t c = cnt - q_first;
            if (c > 0)
                DGC_TRY(sample_strided_launch(vec, s_start + q_first * s_stride, s_stride, c, w.samples + q_first, s));
        }
    }
    return DGC_OK;
}

// K3 threshold over the samples, then the selection (lists kept from begin).
int compress_finish(float* vec, float* mmt, int64_t s_start, int64_t s_stride, int64_t top_k_samples,
                    const dgc_select_params* p, float* spec, float margin, void* values, void* indices,
                    int64_t* count_out, dgc_select_info* info, void* ws, size_t ws_bytes, int sync_mode,
                    hipStream_t s) {
    DGC_TRY(compress_check(p, values, indices, s_start, s_stride, top_k_samples, true));
    if (!vec || (p->masking && !mmt)) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress: null vec/mmt");
    Layout L;
    SelWS w;
    OneTable ot{};
    DGC_TRY(one_ws(p, s_start, s_stride, top_k_samples, spec, ws, ws_bytes, L, w, ot));
    // the table dgc_compress_begin wrote serves as is (the layout does not depend on
    // top_k_samples); K3 gets top_k_samples in its arguments
    DGC_TRY(thresholds(w, L, vec, s, top_k_samples));
    dgc_select_params q = *p;
    // DGCSGDMemory.update fused into the emit (1), or deferred into the next K1 (2)
    q.update_memory = p->update_memory == 2 ? 2 : 1;
    return select_core(vec, mmt, cfg_of(q), L, values, indices, count_out, info, w, 1, sync_mode, margin,
                       p->status_sink, p->order_out, s);
}

// ------------------------------------------------------------------ batch
static int batch_layout(const dgc_batch_desc* b, Layout& L, std::vector<TDesc>& td,
                        std::vector<int32_t> (&bt)[BT_COUNT], std::vector<int32_t>& small) {
    if (!b || b->count < 1 || !b->numel || !b->offset || !b->num_selects || !b->num_samples || !b->top_k_samples ||
        !b->sample_stride)
        DGC_FAIL(DGC_ERR_INVALID, "dgc_batch: null or empty tensor table");
    std::vector<TensorIn> in(b->count);
    int64_t prev_end = 0;
    for (int32_t t = 0; t < b->count; ++t) {
        TensorIn& x = in[t];
        x.n = b->numel[t];
        x.off = b->offset[t];
        x.k = b->num_selects[t];
        x.S = b->num_samples[t];
        x.ks = b->top_k_samples[t];
        x.stride = b->sample_stride[t];
        x.upper_count = (int64_t)std::floor((double)x.k * b->upper_bound);
        x.lower_count = (int64_t)std::ceil(b->lower_bound * (double)x.k);
        x.samples = true;
        if (x.n < 1 || x.k < 1 || x.k > x.n || x.S < 1 || x.S > x.n || x.ks < 1 || x.ks > x.S)
            DGC_FAIL(DGC_ERR_INVALID, "dgc_batch: tensor %d: bad numel/num_selects/num_samples/top_k_samples", t);
        if (b->resample) {
            char who[48];
            std::snprintf(who, sizeof(who), "dgc_batch: tensor %d", t);
            DGC_TRY(check_replay_width(x.n, x.k, who));
        }
        if (x.n != x.S && (x.stride < 4 || x.stride >= (1LL << 30)))
            DGC_FAIL(DGC_ERR_INVALID, "dgc_batch: tensor %d: sample stride %lld outside [4, 2^30)", t,
                     (long long)x.stride);
        if (x.off % kSeg || x.off < prev_end)
            DGC_FAIL(DGC_ERR_INVALID,
                     "dgc_batch: tensor %d: offset %lld must be a multiple of %d, ascending, non-overlapping", t,
                     (long long)x.off, kSeg);
        prev_end = x.off + (int64_t)align_up((size_t)x.n, 4);
        if (prev_end > b->flat_numel) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch: tensor %d past flat_numel", t);
    }
    if (b->int32_indices && b->flat_numel > 2147483647LL)
        DGC_FAIL(DGC_ERR_OVERFLOW, "dgc_batch: int32 indices cannot address %lld elements", (long long)b->flat_numel);
    if (b->dtype != DGC_F32 && b->dtype != DGC_BF16 && b->dtype != DGC_F16)
        DGC_FAIL(DGC_ERR_DTYPE, "dgc_batch: dtype must be DGC_F32, DGC_BF16 or DGC_F16");
    build_layout(in.data(), b->count, true, L, td, bt, small);
    return DGC_OK;
}

// A 16-bit batch (dtype bf16 / fp16) selects on the velocities' fp32 image without
// touching it (update_memory 0; the 16-bit state is masked from the payload,
// dgc_mask_packed16), its wire values in the parameter dtype unless fp16_values, and its
// threshold *= bound products rounded to the dtype.
static SelCfg cfg_of_batch(const dgc_batch_desc* b) {
    const bool half = b->dtype == DGC_BF16 || b->dtype == DGC_F16;
    return SelCfg{(float)b->upper_bound, (float)b->lower_bound, b->max_iters, b->resample, b->momentum_masking,
                  b->fp16_values ? DGC_F16 : (half ? b->dtype : DGC_F32), b->int32_indices ? DGC_I32 : DGC_I64,
                  half ? 0 : (b->deferred_masking ? 2 : 1), half ? b->dtype : DGC_F32,
                  b->resample_order == 1 ? 1 : 0};
}

size_t batch_ws_bytes(const dgc_batch_desc* b) {
    Layout L;
    std::vector<TDesc> td;
    std::vector<int32_t> bt[BT_COUNT];
    std::vector<int32_t> small;
    if (batch_layout(b, L, td, bt, small) != DGC_OK) return 0;
    size_t n = 0;
    carve_select(nullptr, L, &n);
    return n;
}

int batch_init(const dgc_batch_desc* b, void* ws, size_t ws_bytes, hipStream_t s) {
    Layout L;
    std::vector<TDesc> td;
    std::vector<int32_t> bt[BT_COUNT];
    std::vector<int32_t> small;
    DGC_TRY(batch_layout(b, L, td, bt, small));
    size_t need = 0;
    carve_select(nullptr, L, &need);
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_batch_init: workspace needs %zu bytes, 256-B aligned", need);
    SelWS w = carve_select(ws, L);
    DGC_HIP(hipMemsetAsync(w.st, 0, sizeof(SelState) * L.T, s));
    DGC_HIP(hipMemsetAsync(w.setg, 0, sizeof(SetG) * L.T, s));                         // zero at rest
    DGC_HIP(hipMemsetAsync(w.chain, 0, kChainWords * sizeof(uint32_t), s));            // zero at rest
    DGC_HIP(hipMemsetAsync(w.samples, 0, sizeof(float) * L.nsamp, s));   // the window histograms: zero at rest
    DGC_HIP(hipMemcpyAsync(w.td, td.data(), sizeof(TDesc) * L.T, hipMemcpyHostToDevice, s));
    for (int which = 0; which < BT_COUNT; ++which)
        DGC_HIP(hipMemcpyAsync(w.bt[which], bt[which].data(), sizeof(int32_t) * (L.T + 1), hipMemcpyHostToDevice, s));
    if (L.nsmall + L.nwins)
        DGC_HIP(hipMemcpyAsync(w.small, small.data(), sizeof(int32_t) * (L.nsmall + L.nwins), hipMemcpyHostToDevice,
                               s));
    hipLaunchKernelGGL(k_spec_reset, dim3(1), dim3(256), 0, s, w.spec, L.T);
    DGC_LAUNCHED();
    // the host tables are pageable and local: let the copies finish first
    DGC_HIP(hipStreamSynchronize(s));
    return DGC_OK;
}

// Host layout + workspace check shared by the batch entry points.
static int batch_ws(const dgc_batch_desc* b, void* ws, size_t ws_bytes, const char* who, Layout& L,
                    std::vector<TDesc>& td, SelWS& w) {
    std::vector<int32_t> bt[BT_COUNT];
    std::vector<int32_t> small;
    DGC_TRY(batch_layout(b, L, td, bt, small));
    size_t need = 0;
    carve_select(nullptr, L, &need);
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255))
        DGC_FAIL(DGC_ERR_WORKSPACE, "%s: workspace needs %zu bytes, 256-B aligned", who, need);
    w = carve_select(ws, L);
    return DGC_OK;
}

// K1 over every tensor (+ fused strided samples + speculative candidate lists), the
// gradients from the flat buffer (grads == null) or from a host table of T device
// pointers (grads[t]: numel[t] contiguous floats, 16-B aligned).
int batch_compress_begin(const dgc_batch_desc* b, const float* grad, const float* const* grads, float* mmt,
                         float* vec, const int64_t* starts, void* ws, size_t ws_bytes, hipStream_t s) {
    Layout L;
    std::vector<TDesc> td;
    SelWS w;
    DGC_TRY(batch_ws(b, ws, ws_bytes, "dgc_batch_compress", L, td, w));
    if ((!grad && !grads) || !mmt || !vec || !starts) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: null pointer");
    if ((grad && !aligned16(grad)) || !aligned16(mmt) || !aligned16(vec))
        DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: flat buffers must be 16-B aligned");
    if (grads)
        for (int32_t t = 0; t < L.T; ++t)
            if (!grads[t] || !aligned16(grads[t]))
                DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: gradient %d is null or not 16-B aligned", t);
    for (int32_t t = 0; t < L.T; ++t)
        if (td[t].samp_off >= 0 && (starts[t] < 0 || starts[t] >= td[t].stride))
            DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: tensor %d: sample start outside [0, stride)", t);
    // up to 64 starts go to K1 in its arguments; a larger batch puts them first
    StartChunk arg{};
    arg.ptrs = grads ? 1 : 0;
    if (L.T <= 64) {
        arg.count = L.T;
        for (int i = 0; i < L.T; ++i) {
            arg.start[i] = td[i].samp_off >= 0 ? starts[i] : 0;
            arg.grad[i] = grads ? grads[i] : nullptr;
        }
    } else {
        for (int32_t t0 = 0; t0 < L.T; t0 += 64) {
            StartChunk c{};
            c.first = t0;
            c.count = std::min<int32_t>(64, L.T - t0);
            c.ptrs = arg.ptrs;
            for (int i = 0; i < c.count; ++i) {
                c.start[i] = td[t0 + i].samp_off >= 0 ? starts[t0 + i] : 0;
                c.grad[i] = grads ? grads[t0 + i] : nullptr;
            }
            hipLaunchKernelGGL(k_put_starts, dim3(1), dim3(64), 0, s, w, c);
            DGC_LAUNCHED();
        }
    }
    if (L.grid[BT_K1] > 0x7FFFFFFFLL) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: too many segments");
    if (b->nesterov)
        hipLaunchKernelGGL((k_compensate_list<true, false>), dim3((unsigned)L.grid[BT_K1]), dim3(kBlock), 0, s, grad,
                           mmt, vec, b->momentum, w, arg, (int)write_through(L.nseg * kSeg), OneTable{});
    else
        hipLaunchKernelGGL((k_compensate_list<false, false>), dim3((unsigned)L.grid[BT_K1]), dim3(kBlock), 0, s, grad,
                           mmt, vec, b->momentum, w, arg, (int)write_through(L.nseg * kSeg), OneTable{});
    DGC_LAUNCHED();
    return DGC_OK;
}

// K3 thresholds, then the selection of every tensor into the one packed payload.
int batch_compress_finish(const dgc_batch_desc* b, float* mmt, float* vec, void* payload, dgc_select_info* info,
                          void* ws, size_t ws_bytes, int sync_mode, hipStream_t s) {
    Layout L;
    std::vector<TDesc> td;
    SelWS w;
    DGC_TRY(batch_ws(b, ws, ws_bytes, "dgc_batch_compress", L, td, w));
    if (!mmt || !vec || !payload) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: null pointer");
    DGC_TRY(thresholds(w, L, vec, s));
    int64_t cap = 0;
    for (const TDesc& d : td) cap += d.k;
    const SelCfg cfg = cfg_of_batch(b);
    int64_t voff = 0, ioff = 0;
    payload_layout(cap, cfg.vdtype, cfg.idtype, &voff, &ioff);
    char* pl = static_cast<char*>(payload);
    return select_core(vec, mmt, cfg, L, pl + voff, pl + ioff, reinterpret_cast<int64_t*>(pl), info, w, 1,
                       sync_mode, b->spec_margin, b->status_sink, reinterpret_cast<int64_t*>(pl) + 1, s);
}

// The strided samples |x[start + q * stride]| of every sampled tensor from a flat fp32
// buffer (K1 writes them on the fp32 path); grid: (chunks, T).
__global__ void __launch_bounds__(kBlock) k_batch_sample(SelWS w, const float* __restrict__ x_flat) {
    const int t = blockIdx.y;
    const TDesc d = w.td[t];
    if (d.samp_off < 0) return;
    const int64_t start = w.starts[t], cnt = w.scnt[t];
    const float* x = x_flat + d.off + start;
    float* out = w.samples + d.samp_off;
    for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < cnt; q += (int64_t)gridDim.x * kBlock)
        out[q] = fabsf(x[q * d.stride]);
}

// The selection of a batch over a flat fp32 buffer vec32 that no K1 of this library
// produced (a 16-bit batch's velocity image, dgc_compensate16): the strided samples,
// then dgc_batch_compress_finish's thresholds and selection (no candidate lists: the
// first count is a full pass). With dtype = DGC_F32 and update_memory (the desc's
// deferred_masking off) it masks vec32 like the fused path; a 16-bit batch never
// writes vec32.
int batch_select(const dgc_batch_desc* b, float* vec32, float* mmt32, const int64_t* starts, void* payload,
                 dgc_select_info* info, void* ws, size_t ws_bytes, int sync_mode, hipStream_t s) {
    Layout L;
    std::vector<TDesc> td;
    SelWS w;
    DGC_TRY(batch_ws(b, ws, ws_bytes, "dgc_batch_select", L, td, w));
    if (!vec32 || !starts || !payload) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_select: null pointer");
    const SelCfg cfg = cfg_of_batch(b);
    if (cfg.update_memory && cfg.masking && !mmt32) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_select: masking needs mmt");
    for (int32_t t = 0; t < L.T; ++t)
        if (td[t].samp_off >= 0 && (starts[t] < 0 || starts[t] >= td[t].stride))
            DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_select: tensor %d: sample start outside [0, stride)", t);
    for (int32_t t0 = 0; t0 < L.T; t0 += 64) {
        StartChunk c{};
        c.first = t0;
        c.count = std::min<int32_t>(64, L.T - t0);
        for (int i = 0; i < c.count; ++i) c.start[i] = td[t0 + i].samp_off >= 0 ? starts[t0 + i] : 0;
        hipLaunchKernelGGL(k_put_starts, dim3(1), dim3(64), 0, s, w, c);
        DGC_LAUNCHED();
    }
    int64_t smax = 0;
    for (const TDesc& d : td) smax = std::max(smax, d.samp_off >= 0 ? d.S + 1 : 0);
    if (smax > 0) {
        hipLaunchKernelGGL(k_batch_sample, dim3((unsigned)std::min<int64_t>(ceil_div(smax, (int64_t)kBlock), 1024),
                                                (unsigned)L.T), dim3(kBlock), 0, s, w, vec32);
        DGC_LAUNCHED();
    }
    hipLaunchKernelGGL(k_no_lists, dim3(1), dim3(256), 0, s, w);   // t_list = +inf: no K1 lists
    DGC_LAUNCHED();
    DGC_TRY(thresholds(w, L, vec32, s));
    int64_t cap = 0;
    for (const TDesc& d : td) cap += d.k;
    int64_t voff = 0, ioff = 0;
    payload_layout(cap, cfg.vdtype, cfg.idtype, &voff, &ioff);
    char* pl = static_cast<char*>(payload);
    return select_core(vec32, mmt32, cfg, L, pl + voff, pl + ioff, reinterpret_cast<int64_t*>(pl), info, w, 1,
                       sync_mode, b->spec_margin, b->status_sink, reinterpret_cast<int64_t*>(pl) + 1, s);
}

int batch_compress(const dgc_batch_desc* b, const float* grad, float* mmt, float* vec, const int64_t* starts,
                   void* payload, dgc_select_info* info, void* ws, size_t ws_bytes, int sync_mode, hipStream_t s) {
    if (!payload) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress: null pointer");
    DGC_TRY(batch_compress_begin(b, grad, nullptr, mmt, vec, starts, ws, ws_bytes, s));
    return batch_compress_finish(b, mmt, vec, payload, info, ws, ws_bytes, sync_mode, s);
}

int compress_flush(float* vec, float* mmt, int64_t s_stride, const dgc_select_params* p, void* ws, size_t ws_bytes,
                   hipStream_t s) {
    if (!p || !vec) DGC_FAIL(DGC_ERR_INVALID, "dgc_compress_flush: null params/vec");
    Layout L;
    SelWS w;
    OneTable ot{};
    DGC_TRY(one_ws(p, 0, s_stride, 1, nullptr, ws, ws_bytes, L, w, ot));   // tables as the last call left them
    return mask_flush(vec, mmt, L, w, s);
}

int batch_flush(const dgc_batch_desc* b, float* mmt, float* vec, void* ws, size_t ws_bytes, hipStream_t s) {
    Layout L;
    std::vector<TDesc> td;
    std::vector<int32_t> bt[BT_COUNT];
    std::vector<int32_t> small;
    DGC_TRY(batch_layout(b, L, td, bt, small));
    size_t need = 0;
    carve_select(nullptr, L, &need);
    if (!ws || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 255) || !vec || !mmt)
        DGC_FAIL(DGC_ERR_WORKSPACE, "dgc_batch_flush: workspace needs %zu bytes, 256-B aligned", need);
    return mask_flush(vec, mmt, L, carve_select(ws, L), s);
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
    return dgc::one_ws_bytes(numel, num_selects, num_samples, true);
}

extern "C" int dgc_compress_begin(const float* grad, float* mmt, float* vec, float momentum, int32_t nesterov,
                                  int64_t sample_start, int64_t sample_stride, const dgc_select_params* params,
                                  const float* spec_threshold, void* ws, size_t ws_bytes, void* stream) {
    // begin only reads spec[0] (the list threshold); finish updates it
    return dgc::compress_begin(grad, mmt, vec, momentum, nesterov != 0, sample_start, sample_stride, params,
                               const_cast<float*>(spec_threshold), ws, ws_bytes, static_cast<hipStream_t>(stream));
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

extern "C" size_t dgc_batch_workspace(const dgc_batch_desc* batch) { return dgc::batch_ws_bytes(batch); }

extern "C" int dgc_batch_init(const dgc_batch_desc* batch, void* ws, size_t ws_bytes, void* stream) {
    return dgc::batch_init(batch, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_batch_compress(const dgc_batch_desc* batch, const float* grad, float* mmt, float* vec,
                                  const int64_t* sample_starts, void* payload, dgc_select_info* info_out, void* ws,
                                  size_t ws_bytes, int32_t sync_mode, void* stream) {
    return dgc::batch_compress(batch, grad, mmt, vec, sample_starts, payload, info_out, ws, ws_bytes, sync_mode,
                               static_cast<hipStream_t>(stream));
}

extern "C" int dgc_batch_compress_begin(const dgc_batch_desc* batch, const float* grad, float* mmt, float* vec,
                                        const int64_t* sample_starts, void* ws, size_t ws_bytes, void* stream) {
    return dgc::batch_compress_begin(batch, grad, nullptr, mmt, vec, sample_starts, ws, ws_bytes,
                                     static_cast<hipStream_t>(stream));
}

extern "C" int dgc_batch_select(const dgc_batch_desc* batch, float* vec32, float* mmt32, const int64_t* sample_starts,
                                void* payload, dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                                void* stream) {
    return dgc::batch_select(batch, vec32, mmt32, sample_starts, payload, info_out, ws, ws_bytes, sync_mode,
                             static_cast<hipStream_t>(stream));
}

extern "C" int dgc_batch_compress_begin_ptrs(const dgc_batch_desc* batch, const float* const* grads, float* mmt,
                                             float* vec, const int64_t* sample_starts, void* ws, size_t ws_bytes,
                                             void* stream) {
    if (!grads) DGC_FAIL(DGC_ERR_INVALID, "dgc_batch_compress_begin_ptrs: null gradient table");
    return dgc::batch_compress_begin(batch, nullptr, grads, mmt, vec, sample_starts, ws, ws_bytes,
                                     static_cast<hipStream_t>(stream));
}

extern "C" int dgc_batch_compress_finish(const dgc_batch_desc* batch, float* mmt, float* vec, void* payload,
                                         dgc_select_info* info_out, void* ws, size_t ws_bytes, int32_t sync_mode,
                                         void* stream) {
    return dgc::batch_compress_finish(batch, mmt, vec, payload, info_out, ws, ws_bytes, sync_mode,
                                      static_cast<hipStream_t>(stream));
}

#ifdef DGC_K5_PROF
extern "C" int dgc_ce_prof(void* out) {
    DGC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dgc::g_ce_prof), sizeof(dgc::g_ce_prof)));
    return DGC_OK;
}

extern "C" int dgc_es_prof(void* out) {   // tools/es_prof.py
    DGC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dgc::g_es_prof), sizeof(dgc::g_es_prof)));
    return DGC_OK;
}

extern "C" int dgc_pass_prof(void* out) {   // tools/pass_prof.py
    DGC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dgc::g_pass_prof), sizeof(dgc::g_pass_prof)));
    return DGC_OK;
}

extern "C" int dgc_rs_prof(void* out) {   // tools/k3_prof.py
    DGC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dgc::g_rs_prof), sizeof(dgc::g_rs_prof)));
    return DGC_OK;
}

extern "C" int dgc_k5_prof(void* out, int reset) {
    if (reset) {
        dgc::K5Prof z{};
        DGC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dgc::g_k5prof), &z, sizeof(z)));
        return DGC_OK;
    }
    DGC_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dgc::g_k5prof), sizeof(dgc::K5Prof)));
    return DGC_OK;
}
#endif

extern "C" int dgc_compress_flush(float* vec, float* mmt, int64_t sample_stride, const dgc_select_params* params,
                                  void* ws, size_t ws_bytes, void* stream) {
    return dgc::compress_flush(vec, mmt, sample_stride, params, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dgc_batch_flush(const dgc_batch_desc* batch, float* mmt, float* vec, void* ws, size_t ws_bytes,
                               void* stream) {
    return dgc::batch_flush(batch, mmt, vec, ws, ws_bytes, static_cast<hipStream_t>(stream));
}
