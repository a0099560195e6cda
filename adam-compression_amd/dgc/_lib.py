"""ctypes binding of ``libdgc_hip.so`` (the C ABI declared in ``include/dgc_hip.h``).

The product path has no CPU fallback: if the library cannot be loaded, or a tensor
is not a float tensor on an MI355X (fp32; bf16 / fp16 on the per-tensor path), every
entry point raises.
"""
import ctypes
import os

import torch

__all__ = ["lib", "check", "stream_of", "ptr", "SelectParams", "SelectInfo", "Workspace",
           "VD", "ID", "BRANCHES", "LIB_PATH", "available", "BatchDesc"]

LIB_PATH = os.environ.get(
    "DGC_HIP_LIB",
    os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libdgc_hip.so"))

DGC_OK = 0
# speculative list threshold after a miss = SPEC_MARGIN x the predicted final threshold
# (dgc_hip.h, spec_threshold); DGC_SPEC_MARGIN overrides it for A/B runs (results are
# identical: it only chooses how much K1 lists ahead)
SPEC_MARGIN = float(os.environ.get("DGC_SPEC_MARGIN", "0.8"))
SYNC_DEVICE, SYNC_HOST = 0, 1
VD = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2}
HALF = (torch.bfloat16, torch.float16)   # 16-bit parameters (dgc_*16 entry points)
ID = {torch.int64: 0, torch.int32: 1}
BRANCHES = {0: "direct", 1: "ok", 2: "trunc", 3: "resample", 4: "exhausted"}
TIE_RULES = {0: "none", 1: "exact", 2: "set"}


class SelectParams(ctypes.Structure):
    _fields_ = [("numel", ctypes.c_int64), ("num_selects", ctypes.c_int64),
                ("num_samples", ctypes.c_int64), ("upper_count", ctypes.c_int64),
                ("lower_count", ctypes.c_int64), ("upper", ctypes.c_float), ("lower", ctypes.c_float),
                ("max_iters", ctypes.c_int32), ("resample", ctypes.c_int32), ("masking", ctypes.c_int32),
                ("vdtype", ctypes.c_int32), ("idtype", ctypes.c_int32), ("update_memory", ctypes.c_int32),
                ("thr_dtype", ctypes.c_int32), ("resample_order", ctypes.c_int32),
                ("status_sink", ctypes.c_void_p), ("order_out", ctypes.c_void_p)]


class SelectInfo(ctypes.Structure):
    _fields_ = [("count", ctypes.c_int64), ("candidates", ctypes.c_int64),
                ("threshold0", ctypes.c_float), ("threshold", ctypes.c_float),
                ("branch", ctypes.c_int32), ("recounts", ctypes.c_int32),
                ("overflow_segments", ctypes.c_int32), ("full_passes", ctypes.c_int32),
                ("tie_rule", ctypes.c_int32), ("window_keys", ctypes.c_int32),
                ("k5_status", ctypes.c_int32), ("list_threshold", ctypes.c_float)]


K5_FALLBACK, K5_BROKEN, K5_RECOVERED, K5_SET_FALLBACK, K5_SET_BROKEN = 1, 2, 4, 8, 16


def info_dict(i, what):
    """A dgc_select_info record as the engines report it; raises when the resample
    replay's multi-workgroup phase broke (its selection would not be the reference's)."""
    if i.k5_status & K5_BROKEN:
        raise RuntimeError(f"{what}: the resample replay's multi-workgroup phase timed out at a barrier after it "
                           "started (workgroups not co-resident?); this step's selection is not reliable")
    return dict(count=i.count, candidates=i.candidates, threshold0=i.threshold0, threshold=i.threshold,
                branch=BRANCHES.get(i.branch, i.branch), recounts=i.recounts,
                overflow_segments=i.overflow_segments, full_passes=i.full_passes,
                tie_rule=TIE_RULES.get(i.tie_rule, i.tie_rule), window_keys=i.window_keys,
                list_threshold=i.list_threshold,
                k5_fallback=bool(i.k5_status & K5_FALLBACK), k5_recovered=bool(i.k5_status & K5_RECOVERED),
                k5s_fallback=bool(i.k5_status & K5_SET_FALLBACK), k5s_broken=bool(i.k5_status & K5_SET_BROKEN))


INFO_BYTES = ctypes.sizeof(SelectInfo)


# every sink's pinned words stay allocated for the life of the process: the library
# holds their addresses (dgc_select_params.status_sink, dgc_decompress_bind_sink)
_SINK_WORDS = []


def _unbind(ws_ptr):
    if _lib is not None:
        _lib.dgc_decompress_bind_sink(ctypes.c_void_p(ws_ptr), None)


class StatusSink:
    """The engines' per-step error check without a host synchronisation: four pinned
    host int32 words the kernels write only when something is wrong —

      [0] the selection's finish: its k5_status when a resample replay broke
          (DGC_K5_BROKEN; ``status_sink``)
      [1] decompress: an index outside the output (1: dropped; the reference's
          ``index_put_`` raises, dgc/compression.py:191); the 16-bit decompress also
          stores 2 here for a bad header count
      [2] decompress: a gathered header count outside [0, capacity] (a corrupted
          payload, the reference's "allgathered data are random data" README.md:132)
      [3] DGCSGDMemory.update: an index outside [-n, n) (the reference's
          ``index_fill_`` raises, dgc/memory.py:76-77)

    ``bind(ws)`` routes a decompress workspace's error bits into words [1, 2]
    (``dgc_decompress_bind_sink``); ``index_flag`` is word [3]'s address, passed as a
    kernel's ``bad_flag``. ``check()`` reads the words — free — and raises once one is
    set, i.e. at the first step the host issues after the GPU finished the bad call (a
    host that runs ahead of the GPU sees it that many steps later; ``check(sync=True)``
    waits for the stream first). A reported decompress / masking error is cleared, so a
    caller that catches it can go on."""

    def __init__(self, what, device):
        self.what = what
        self.device = device
        self.word = torch.zeros(4, dtype=torch.int32, pin_memory=torch.cuda.is_available())
        _SINK_WORDS.append(self.word)
        self._view = self.word.numpy()   # the same host words, read without a tensor op

    @property
    def address(self):
        return self.word.data_ptr()

    @property
    def decompress_words(self):
        return self.word.data_ptr() + 4

    @property
    def index_flag(self):
        return self.word.data_ptr() + 12

    def bind(self, ws):
        """Routes the decompress workspace tensor ``ws``'s error bits here (unbound when
        ``ws`` is freed)."""
        import weakref
        check(lib().dgc_decompress_bind_sink(ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(self.decompress_words)),
              "dgc_decompress_bind_sink")
        weakref.finalize(ws, _unbind, ws.data_ptr())
        return ws

    def check(self, sync=False):
        if sync:
            torch.cuda.current_stream(self.device).synchronize()
        v = self._view
        k5 = int(v[0])
        if k5 & K5_BROKEN:
            raise RuntimeError(f"{self.what}: the resample replay's multi-workgroup phase timed out at a barrier after "
                               f"it started (k5_status {k5}; workgroups not co-resident?); the selection of that step "
                               "is not reliable")
        if v[1] or v[2] or v[3]:
            why = []
            if v[1] & 1:
                why.append("a decompressed index was outside the gradient (its entry was dropped)")
            if v[2] or v[1] & 2:
                why.append("a gathered payload header held a count outside [0, capacity] (the run was clamped)")
            if v[3]:
                why.append("DGCSGDMemory.update got an index outside the state (not masked)")
            v[1:] = 0
            raise RuntimeError(f"{self.what}: " + "; ".join(why) + " — a foreign or corrupted payload (the reference's "
                               "index_put_ / index_fill_ raise IndexError here)")


class BatchDesc(ctypes.Structure):
    """dgc_batch_desc (include/dgc_hip.h): a batch's tensors and shared settings."""
    _fields_ = [("count", ctypes.c_int32), ("numel", ctypes.POINTER(ctypes.c_int64)),
                ("offset", ctypes.POINTER(ctypes.c_int64)), ("num_selects", ctypes.POINTER(ctypes.c_int64)),
                ("num_samples", ctypes.POINTER(ctypes.c_int64)), ("top_k_samples", ctypes.POINTER(ctypes.c_int64)),
                ("sample_stride", ctypes.POINTER(ctypes.c_int64)), ("flat_numel", ctypes.c_int64),
                ("upper_bound", ctypes.c_double), ("lower_bound", ctypes.c_double),
                ("max_iters", ctypes.c_int32), ("resample", ctypes.c_int32), ("momentum_masking", ctypes.c_int32),
                ("fp16_values", ctypes.c_int32), ("int32_indices", ctypes.c_int32), ("nesterov", ctypes.c_int32),
                ("momentum", ctypes.c_float), ("spec_margin", ctypes.c_float),
                ("deferred_masking", ctypes.c_int32), ("dtype", ctypes.c_int32),
                ("resample_order", ctypes.c_int32), ("status_sink", ctypes.c_void_p)]

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_F = ctypes.c_float
_SZ = ctypes.c_size_t

_SIGNATURES = {
    "dgc_last_error": (ctypes.c_char_p, []),
    "dgc_version": (ctypes.c_char_p, []),
    "dgc_compensate": (ctypes.c_int, [_P, _P, _P, _P, _I64, _F, _I32, _I32, _P, _I64, _I64, _I64, _P]),
    "dgc_mask_indices": (ctypes.c_int, [_P, _P, _I64, _P, _I32, _I64, _P, _P]),
    "dgc_sample_strided": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I64, _P]),
    "dgc_sample_gather": (ctypes.c_int, [_P, _P, _I64, _P, _P]),
    "dgc_kth_largest_workspace": (_SZ, [_I64]),
    "dgc_kth_largest": (ctypes.c_int, [_P, _I64, _I64, _P, _P, _SZ, _P]),
    "dgc_select_workspace": (_SZ, [_I64, _I64]),
    "dgc_select": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(SelectParams), _P, _P, _P, _P, _P, _SZ,
                                  _I32, _P]),
    "dgc_compress_workspace": (_SZ, [_I64, _I64, _I64]),
    "dgc_compress": (ctypes.c_int, [_P, _P, _P, _F, _I32, _I64, _I64, _I64, ctypes.POINTER(SelectParams),
                                    _P, _F, _P, _P, _P, _P, _P, _SZ, _I32, _P]),
    "dgc_compress_begin": (ctypes.c_int, [_P, _P, _P, _F, _I32, _I64, _I64, ctypes.POINTER(SelectParams), _P, _P,
                                          _SZ, _P]),
    "dgc_compress_finish": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, ctypes.POINTER(SelectParams), _P, _F, _P, _P,
                                           _P, _P, _P, _SZ, _I32, _P]),
    "dgc_compress_flush": (ctypes.c_int, [_P, _P, _I64, ctypes.POINTER(SelectParams), _P, _SZ, _P]),
    "dgc_decompress_workspace": (_SZ, [_I64, _I32]),
    "dgc_decompress_packed_workspace": (_SZ, [_I64, _I32, _I64]),
    "dgc_decompress": (ctypes.c_int, [_P, _I32, _P, _I32, _I64, ctypes.POINTER(ctypes.c_int64), _I32, _P,
                                      _I64, _F, _P, _SZ, _P]),
    "dgc_payload_layout": (_I64, [_I64, _I32, _I32, ctypes.POINTER(ctypes.c_int64),
                                  ctypes.POINTER(ctypes.c_int64)]),
    "dgc_decompress_packed": (ctypes.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _P, _I64, _F, _P, _SZ, _P]),
    "dgc_scatter_packed": (ctypes.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _P, _I64, _F, _P, _SZ, _P]),
    "dgc_decompress_packed_over": (ctypes.c_int, [_P, _P, _I32, _I64, _I64, _I32, _I32, _P, _I64, _F, _P, _SZ, _P]),
    "dgc_clear_packed": (ctypes.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _P, _I64, _P, _SZ, _P]),
    "dgc_scatter_packed_cleared": (ctypes.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _P, _I64, _F, _P, _SZ, _P]),
    "dgc_payload_split_layout": (_I64, [_I64, _I32, _I32, _I32, _P]),
    "dgc_payload_split_bytes": (_I64, [_I64, _I32, _I32, _I32]),
    "dgc_payload_split": (ctypes.c_int, [_P, _I64, _I32, _I32, _I32, _P, _P]),
    "dgc_decompress_split_workspace": (_SZ, [_I64, _I32, _I32, _I64]),
    "dgc_scatter_split": (ctypes.c_int, [_P, _I32, _I32, _I32, _I64, _I32, _I32, _P, _I64, _F, _I32, _P, _SZ, _P]),
    "dgc_clear_split": (ctypes.c_int, [_P, _I32, _I32, _I64, _I32, _I32, _P, _I64, _P, _SZ, _P]),
    "dgc_fill_zero": (ctypes.c_int, [_P, _I64, _P]),
    "dgc_decompress_status": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32), _P]),
    "dgc_decompress_bind_sink": (ctypes.c_int, [_P, _P]),
    "dgc_batch_workspace": (_SZ, [ctypes.POINTER(BatchDesc)]),
    "dgc_batch_init": (ctypes.c_int, [ctypes.POINTER(BatchDesc), _P, _SZ, _P]),
    "dgc_batch_compress": (ctypes.c_int, [ctypes.POINTER(BatchDesc), _P, _P, _P, ctypes.POINTER(_I64), _P, _P, _P,
                                          _SZ, _I32, _P]),
    "dgc_batch_compress_begin": (ctypes.c_int, [ctypes.POINTER(BatchDesc), _P, _P, _P, ctypes.POINTER(_I64), _P,
                                                _SZ, _P]),
    "dgc_batch_compress_begin_ptrs": (ctypes.c_int, [ctypes.POINTER(BatchDesc), ctypes.POINTER(_P), _P, _P,
                                                     ctypes.POINTER(_I64), _P, _SZ, _P]),
    "dgc_gather_cast": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.POINTER(_I64), _I32, _P, _I32,
                                       _P]),
    "dgc_compensate_wire": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _I64, _F, _I32, _P]),
    "dgc_compensate_wire_avg": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _I64, _F, _I32, _P]),
    "dgc_compensate_multi": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.POINTER(_I64), _I32,
                                            _I32, _P, _P, _F, _I32, _P]),
    "dgc_rank_sum": (ctypes.c_int, [_P, _I32, _I32, _I64, _I64, _I32, _P, _P]),
    "dgc_compensate_ranks": (ctypes.c_int, [_P, _I32, _I32, _I64, _P, _P, _I64, _F, _I32, _P]),
    "dgc_batch_select": (ctypes.c_int, [ctypes.POINTER(BatchDesc), _P, _P, ctypes.POINTER(_I64), _P, _P, _P, _SZ, _I32,
                                         _P]),
    "dgc_mask_packed16": (ctypes.c_int, [_P, _I64, _I32, _I32, _P, _P, _I64, _P]),
    "dgc_decompress_packed16": (ctypes.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _P, _I32, _I64, _F, _P, _P]),
    "dgc_gather16": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.POINTER(_I64), _I32, _P, _P]),
    "dgc_batch_compress_finish": (ctypes.c_int, [ctypes.POINTER(BatchDesc), _P, _P, _P, _P, _P, _SZ, _I32, _P]),
    "dgc_batch_flush": (ctypes.c_int, [ctypes.POINTER(BatchDesc), _P, _P, _P, _SZ, _P]),
    "dgc_hbm_probe": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _P]),
    "dgc_compensate16": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _F, _I32, _I32, _I32, _P]),
    "dgc_mask_indices16": (ctypes.c_int, [_P, _P, _I64, _P, _I32, _I64, _P, _P]),
    "dgc_widen16": (ctypes.c_int, [_P, _P, _I64, _I32, _P]),
    "dgc_decompress16": (ctypes.c_int, [_P, _I32, _P, _I32, ctypes.POINTER(ctypes.c_int64), _I32, _P, _I32, _I64,
                                        _F, _P, _P]),
    "dgc_sgd_step": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P),
                                    ctypes.POINTER(_I64), ctypes.POINTER(_I32), _I32, _F, _F, _F, _F, _I32, _P]),
    "dgc_sgd_step16": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P),
                                      ctypes.POINTER(_I64), ctypes.POINTER(_I32), _I32, _F, _F, _F, _F, _I32, _I32,
                                      _P]),
}

_lib = None
_load_error = None


def _load():
    global _lib, _load_error
    if _lib is not None or _load_error is not None:
        return _lib
    try:
        handle = ctypes.CDLL(LIB_PATH)
        # DGC_LIB_PARTIAL=1 (same-box A/B against an older build, tools/ab_bench.py):
        # symbols the older library lacks stay unbound instead of failing the load
        partial = os.environ.get("DGC_LIB_PARTIAL") == "1"
        for name, (res, args) in _SIGNATURES.items():
            if partial and not hasattr(handle, name):
                continue
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    except OSError as e:   # pragma: no cover - reported through lib()
        _load_error = e
    return _lib


_glue = None


def glue():
    """The batched optimizer's host glue (csrc/glue.cpp, lib/_dgc_glue.so: p.grad pointer
    tables and rebinding over torch's tensor objects); raises if it was not built."""
    global _glue
    if _glue is None:
        import importlib.util
        path = os.path.join(os.path.dirname(LIB_PATH), "_dgc_glue.so")
        if not os.path.exists(path):
            path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "_dgc_glue.so")
        try:
            spec = importlib.util.spec_from_file_location("_dgc_glue", path)
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
        except (ImportError, OSError, AttributeError) as e:
            raise RuntimeError(f"{path} could not be loaded ({e}); build it with `make -C adam-compression_amd/csrc`")
        _glue = mod
    return _glue


def available():
    return _load() is not None


def lib():
    """The loaded library; raises if it is missing (there is no fallback path)."""
    handle = _load()
    if handle is None:
        raise RuntimeError(f"libdgc_hip.so could not be loaded from {LIB_PATH}: {_load_error}. "
                           "Build it with `make -C adam-compression_amd/csrc` (hipcc, gfx950).")
    return handle


def check(status, what="dgc"):
    if status != DGC_OK:
        msg = lib().dgc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def require_cuda_float(t, what, contiguous=True):
    """A contiguous fp32, bf16 or fp16 tensor on the MI355X (the per-tensor path takes all
    three; the engines take fp32 only: require_cuda_f32). Returns its dtype."""
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError(f"{what}: the DGC hot path runs on the MI355X only (got a "
                           f"{'CPU' if torch.is_tensor(t) else type(t).__name__} tensor)")
    if t.dtype not in (torch.float32,) + HALF:
        raise NotImplementedError(f"{what}: fp32, bf16 or fp16 tensors only (got {t.dtype})")
    if contiguous and not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")
    return t.dtype


def require_cuda_f32(t, what):
    if not (torch.is_tensor(t) and t.is_cuda):
        raise RuntimeError(f"{what}: the DGC hot path runs on the MI355X only (got a "
                           f"{'CPU' if torch.is_tensor(t) else type(t).__name__} tensor)")
    if t.dtype != torch.float32:
        raise NotImplementedError(f"{what}: fp32 tensors only (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{what}: tensor must be contiguous")


class Workspace:
    """Grow-only device scratch buffers keyed by (device, tag): the library never allocates.
    Zero-filled when (re)allocated: a compress workspace carries state between calls."""

    def __init__(self):
        self._bufs = {}

    def get(self, device, nbytes, tag="ws"):
        key = (str(device), tag)
        buf = self._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self._bufs[key] = buf
        return buf
