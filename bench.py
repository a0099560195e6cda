#!/usr/bin/env python3
"""DGC hot-path benchmark on MI355X: compensate -> compress (sample, threshold,
select, adaptation, masking) -> RCCL allgather -> decompress, all on the device.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--no-cpu]
    torchrun --nproc-per-node N ... bench.py --gpus N ...

Workloads (BASELINE.json configs; synthetic data of their shapes):
  flat-1B       (default) 1e9-element fp32 bucket, ratio 0.001, nesterov, fp32/int64  [configs[3]]
  flat-7B-bf16  7e9 elements, bf16-origin gradients, ratio 1e-4, int64 indices        [configs[4]]
  resnet50      the 161 gradient tensors of ResNet-50 (54 compressed, 25.5M elements;
                107 dense), ratio 0.001, fp32/int64, one batched step                  [configs[1]]
  vgg16_bn      the 58 gradient tensors of VGG-16-BN (16 compressed, 138.3M elements),
                ratio 0.001, fp16 values / int32 indices                               [configs[2]]

Rank 0 prints ONE JSON line. ``value`` = gradient elements processed by all ranks per
second (each rank compresses its own replica's gradients: weak scaling). ``roofline``
is for the dominant kernel, K1 (compensate + fused sample + candidate lists), timed
with HIP events on the stream it runs on; ``step_hbm`` is the whole step's algorithmic
HBM rate. With ``--gpus N`` and no torchrun, N ranks are spawned on 127.0.0.1.
"""
import argparse
import contextlib
import ctypes
import io
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "adam-compression_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "grad elements/s per DGC step (HBM GB/s % of peak), 0.1% ratio, 1-8 GPUs"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_COPY_GBS = 6290.0            # measured float4 copy ceiling (same guide)
XGMI_LINK_GBS = 153.0            # per link, per direction

# Synthetic gradients: a fresh N(0, 1) gradient per rank and step, seed
# 0xD6C + 1000 * rank + step (torch.randn on the device, generated before the timed
# region), the sample starts from random.Random(42) — except flat-7B-bf16, whose 28 GB
# buffers allow two (steps alternate between seeds 0xD6C + 1000 * rank + {0, 1}).
WORKLOADS = {
    "flat-1B": dict(kind="flat", numel=10 ** 9, ratio=1e-3, grad="normal", nesterov=True,
                    config="BASELINE configs[3]: synthetic 1B-element flat gradient bucket"),
    "flat-7B-bf16": dict(kind="flat", numel=7 * 10 ** 9, ratio=1e-4, grad="bf16", nesterov=True, buffers=2,
                         config="BASELINE configs[4]: synthetic 7B-element bf16-origin gradient"),
    "resnet50": dict(kind="model", model="resnet50", ratio=1e-3, fp16=False, int32=False, nesterov=False,
                     config="BASELINE configs[1]: ResNet-50 ImageNet gradient set"),
    "vgg16_bn": dict(kind="model", model="vgg16_bn", ratio=1e-3, fp16=True, int32=True, nesterov=False,
                     config="BASELINE configs[2]: VGG-16-BN gradient set"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="flat-1B", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-numel", type=float, default=1e9,
                    help="CPU baseline (all cores), flat: elements per step (default: the whole 1B bucket)")
    ap.add_argument("--cpu-numel-1t", type=float, default=5e7, help="CPU-baseline sample (1 thread), flat")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--inputs", default="per-step", choices=["per-step", "alternating"],
                    help="per-step: a fresh gradient per rank and step (SURVEY.md §8d, the headline); alternating: "
                         "two buffers per rank, steps alternating between them (rounds 1-5's input model)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--rccl-one-rank", action="store_true",
                    help="N=1: exchange through a one-rank RCCL group as at N > 1 (the allgather path and its "
                         "timing executed on a one-GPU box); not the headline configuration")
    ap.add_argument("--phases", action="store_true", help="HIP events around every phase (adds markers)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the dense-fill pass and (W = 1) the drop-in DistributedOptimizer comparison")
    ap.add_argument("--dropin-model", default="resnet50", choices=["resnet50", "vgg16_bn"],
                    help="model set of the drop-in comparison of a flat workload's run")
    ap.add_argument("--fill", default="sparse", choices=["inline", "allgather", "sparse"],
                    help="decompress zero_(): sparse = re-zero only the previous step's entries of the bench's "
                         "persistent output (the bench owns it and never writes it; dgc/bucket.py)")
    return ap.parse_args()


# ---------------------------------------------------------------------------- CPU baseline
def cpu_cores():
    """The host cores this process may use: its affinity set, capped by OMP_NUM_THREADS
    when the host sets it (the GPU box exposes every CPU of the machine to affinity but
    grants each job a share, 16, through OMP_NUM_THREADS)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(run, wl, numel, steps, threads):
    """The reference op sequence restated on torch CPU (oracle/torch_cpu.py, pinned to
    the reference's golden fixtures), timed on this host (rank 0, N=1 only) with the GPU
    run's OWN inputs: the gradients of its first ``steps + 1`` steps copied back from
    HBM before the timing (model sets: every compressed tensor; flat buckets: the first
    ``numel`` elements — all of flat-1B's by default), the same sample starts
    (``random.Random(42)`` in the GPU engines' order), one warm-up step, then ``steps``
    timed steps."""
    from oracle import torch_cpu
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    import random
    rng = random.Random(42)
    try:
        if wl["kind"] == "model":
            b = run.b
            host = [run.grad_of(i)[0].cpu() for i in range(steps + 1)]
            tensors = []
            for off, n in zip(b.offsets, b.numels):
                attrs = torch_cpu.attributes(n, wl["ratio"])
                tensors.append((attrs, [g[off: off + n] for g in host], torch.zeros(n), torch.zeros(n),
                                torch.empty(n)))
            N = sum(t[0][0] for t in tensors)

            def step(i):
                for attrs, gs, m, v, out in tensors:   # DGCBatch.draw_starts' order
                    start = rng.randint(0, attrs[4] - 1) if attrs[0] != attrs[2] else 0
                    torch_cpu.cpu_step(gs[i], m, v, out, attrs, start, nesterov=wl["nesterov"])
            what = f"all {len(tensors)} compressed tensors ({N} elements) of {wl['model']}"
        else:
            N = int(min(numel, run.N))
            attrs = torch_cpu.attributes(N, wl["ratio"])
            host = [run.grad_of(i)[:N].cpu() for i in range(steps + 1)]
            m, v, out = torch.zeros(N), torch.zeros(N), torch.empty(N)

            def step(i):
                torch_cpu.cpu_step(host[i], m, v, out, attrs, rng.randint(0, attrs[4] - 1), nesterov=wl["nesterov"])
            what = (f"the whole {N}-element bucket" if N == run.N else
                    f"the first {N} elements of the {run.N}-element bucket (same ratio, sample stride {attrs[4]})")
        step(0)   # warm-up
        t0 = time.perf_counter()
        for i in range(steps):
            step(i + 1)
        dt = (time.perf_counter() - t0) / steps
    finally:
        torch.set_num_threads(prev)
    return {"value": N / dt, "unit": "grad elements/s", "cores": threads, "kind": "port",
            "sample": f"{what}, the GPU run's gradients of steps 1..{steps} after step 0 as warm-up, sample "
                      f"starts from random.Random(42) (compensate+sparsify+update+decompress, W=1, torch "
                      f"{torch.__version__} CPU ops as the reference issues them): {dt * 1e3:.1f} ms/step on "
                      f"{threads} thread(s); {cpu_model()}"}


# ---------------------------------------------------------------------------- profiles
def pmc_traffic(workload, kernel_key="k_compensate_list"):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC profile
    of this exact bench command (tools/pmc_json.py over separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE x2 for gfx950's half count of wide reads)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "round*", f"pmc_{workload}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    for k, v in d.get("kernels", {}).items():
        if kernel_key in k:
            return v["hbm_bytes_per_launch"], os.path.relpath(files[-1], REPO)
    return None, None


def rocprof_k1_ms(workload, kernel_key="k_compensate_list"):
    """The dominant kernel's average duration in the committed rocprofv3 kernel-trace
    stats of this exact bench command (profiles/round*/kstats_<workload>.json): over the
    launches after the warmup (timed_avg_ms) when the trace gave them."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "round*", f"kstats_{workload}.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    for k, v in d.items():
        if kernel_key in k:
            return v.get("timed_avg_ms", v["avg_ms"]), os.path.relpath(files[-1], REPO)
    return None, None


# ---------------------------------------------------------------------------- launcher
def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus, environ):
    """How ``bench.py --gpus N`` runs: None when this process is one rank already
    (torchrun set WORLD_SIZE, or N == 1), else the environments of N child ranks to
    spawn on 127.0.0.1. Raises SystemExit when --gpus disagrees with WORLD_SIZE."""
    if "WORLD_SIZE" in environ:
        world = int(environ["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; they must agree")
        return None
    if gpus <= 1:
        return None
    port = str(free_port())
    envs = []
    for r in range(gpus):
        env = dict(environ)
        env.update(WORLD_SIZE=str(gpus), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        envs.append(env)
    return envs


def check_devices(gpus, devices):
    """Fails fast, before any rank is spawned or touches the GPU, when this node has
    fewer devices than ranks (torch.cuda.device_count() does not initialise HIP)."""
    if devices < gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} needs {gpus} visible GPUs, this node shows {devices} "
                         f"(torch.cuda.device_count()); nothing was launched")


def spawn(envs):
    """One child process per rank (started before this process touches the GPU);
    returns the first non-zero exit code, or 0."""
    import subprocess
    procs = [subprocess.Popen([sys.executable] + sys.argv, env=e) for e in envs]
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c != 0), 0)


# ---------------------------------------------------------------------------- workloads
def gradient_seed(rank, step):
    """the synthetic gradient of ``rank`` at ``step``."""
    return 0xD6C + 1000 * rank + step


def fill_gradient(g, seed, bf16=False, chunk=1 << 30):
    """g = N(0, 1) from one generator seeded ``seed``, in 2^30-element chunks (bf16-rounded
    for the bf16-origin workload: dense ties)."""
    gen = torch.Generator(device=g.device)
    gen.manual_seed(seed)
    for c0 in range(0, g.numel(), chunk):
        c1 = min(g.numel(), c0 + chunk)
        x = torch.randn(c1 - c0, generator=gen, device=g.device)
        g[c0:c1] = x.to(torch.bfloat16).float() if bf16 else x
        del x
    return g


def buffers_that_fit(nsteps, nbytes, dev, reserve):
    """How many per-step gradient buffers of ``nbytes`` fit in the free HBM beside
    ``reserve`` bytes still to be allocated (at least 2; steps cycle through them)."""
    free, _ = torch.cuda.mem_get_info(dev)
    return max(2, min(nsteps, int((free - reserve) // nbytes)))


class FlatRun:
    """One flat bucket per rank through dgc.bucket.DGCBucket; one gradient per step
    (``nsteps`` buffers, generated before timing), or the workload's fixed ``buffers``."""

    def __init__(self, wl, rank, world, dev, fill, nsteps=2):
        from dgc.bucket import DGCBucket
        N = wl["numel"]
        self.N = N
        self.b = DGCBucket(N, compress_ratio=wl["ratio"], momentum=0.9, nesterov=wl["nesterov"], device=dev,
                           world_size=world, fill=fill)
        self.out = torch.empty(N, device=dev)
        want = wl.get("buffers", nsteps)
        self.nbuf = buffers_that_fit(want, 4 * N, dev, reserve=8 << 30) if "buffers" not in wl else want
        self.grads = [fill_gradient(torch.empty(N, device=dev), gradient_seed(rank, s), wl["grad"] == "bf16")
                      for s in range(self.nbuf)]
        self.elements = N
        self.k, self.S = self.b.k, self.b.num_samples
        self.payload = self.b.rank_stride
        self.vbytes, self.ibytes = 4, 8

    def grad_of(self, i):
        return self.grads[i % self.nbuf]

    def step(self, i, ev=None):
        self.b.step(self.grad_of(i), self.out, ev)

    def k1_bytes(self):
        return 20 * self.N + 4 * self.b.cnt    # read g, mmt, vec; write mmt, vec; write the samples

    def probe_buffers(self):
        return [self.grads[0], self.grads[1], self.out], [self.b._mmt, self.b._vec]

    def info(self):
        return self.b.last_info()

    def records(self):
        return [self.b.last_info()]

    def config(self):
        b = self.b
        return {"numel": self.N, "num_selects": b.k, "num_samples": b.num_samples, "sample_stride": b.stride,
                "fill": b.fill, "exchange_parts": b.parts}


def model_gradients(b, n_dense, seed, dev):
    """A model set's gradients of one step: (flat compressed gradients in ``b``'s layout,
    dense gradients), N(0, 1) x 1e-3 tensor after tensor from one generator."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    g = torch.zeros(b.flat_numel, device=dev)
    for off, n in zip(b.offsets, b.numels):
        g[off: off + n] = torch.randn(n, generator=gen, device=dev) * 1e-3
    return g, torch.randn(n_dense, generator=gen, device=dev) * 1e-3


class ModelRun:
    """A model's gradient set per rank: the compressed tensors through one DGCBatch
    step, the dense (dim <= 1) tensors as one flat allreduce + compensate(accumulate=False)
    (dgc/compression.py:173-177, 195-198)."""

    def __init__(self, wl, rank, world, dev, fill="sparse", nsteps=2):
        from dgc import comm, workloads
        from dgc.batch import DGCBatch
        comp, dense = workloads.split(getattr(workloads, wl["model"])())
        self.n_dense = sum(workloads.numel(s) for _, s in dense)
        wire_dt = torch.float16 if wl["fp16"] else torch.float32
        self.exchanging = world > 1 or comm.one_rank_collectives()
        # W > 1: the dense wire values ride in the tail of the packed payload (one allgather)
        extra = self.n_dense * torch.empty(0, dtype=wire_dt).element_size() if self.exchanging else 0
        self.b = DGCBatch(comp, compress_ratio=wl["ratio"], momentum=0.9, nesterov=wl["nesterov"],
                          fp16_values=wl["fp16"], int32_indices=wl["int32"], device=dev, world_size=world, seed=42,
                          fill="inline" if fill in ("inline", "allgather") else "sparse", payload_extra=extra)
        self.n_comp = sum(self.b.numels)
        self.world = world
        # one gradient set per step (x1e-3): every compressed tensor in the batch's flat
        # layout, then the dense tensors, from one generator seeded gradient_seed(rank, step)
        self.nbuf = buffers_that_fit(nsteps, 4 * (self.b.flat_numel + self.n_dense), dev, reserve=2 << 30)
        self.grads = [model_gradients(self.b, self.n_dense, gradient_seed(rank, s), dev) for s in range(self.nbuf)]
        self.dense_mmt = torch.zeros(self.n_dense, device=dev)
        self.dense_out = torch.empty(self.n_dense, device=dev)
        self.wire_dt = wire_dt
        self.dense_wire = self.dense_gathered = None
        if self.exchanging and self.b.extra_off is None:   # split exchange: the dense values on their own
            self.dense_wire = torch.empty(extra, dtype=torch.uint8, device=dev)
            self.dense_gathered = torch.empty(world * extra, dtype=torch.uint8, device=dev)
        self._one = (ctypes.c_int64 * 1)(self.n_dense), (ctypes.c_int64 * 1)(0)
        self.elements = self.n_comp + self.n_dense
        self.k, self.S = self.b.capacity, sum(a[1] for a in self.b.attrs)
        self.payload = self.b.rank_stride
        self.vbytes, self.ibytes = (2 if wl["fp16"] else 4), (4 if wl["int32"] else 8)
        self.nesterov = wl["nesterov"]
        from dgc import _lib
        self._lib = _lib

    def grad_of(self, i):
        return self.grads[i % self.nbuf]

    def step(self, i, ev=None):
        g, gd = self.grad_of(i)
        ev = ev or {}
        L, b = self._lib.lib(), self.b
        from dgc import comm
        b.grad_flat = g   # the model's gradients live in the batch's flat buffer (p.grad views)
        st = self._lib.stream_of(g.device)
        wt = self._lib.VD[self.wire_dt]
        handle = []

        def select():
            b.select()
            if self.exchanging:
                # dense tensors: the fp16 wire cast (dgc/compression.py:173-177) into the
                # payload's tail, exchanged by the same allgather
                src = (ctypes.c_void_p * 1)(gd.data_ptr())
                own = self.dense_wire
                dst = own.data_ptr() if own is not None else b.payload.data_ptr() + b.extra_off
                self._lib.check(L.dgc_gather_cast(src, self._one[0], self._one[1], 1, ctypes.c_void_p(dst), wt, st),
                                "dgc_gather_cast")
                if own is not None:
                    handle.append(comm.allgather_packed_async(own, out=self.dense_gathered))

        for name, fn in (("compensate", b.compensate), ("select", select), ("allgather", b.exchange),
                         ("decompress", b.decompress)):
            pair = ev.get(name)
            if pair:
                pair[0].record()
            fn()
            if pair:
                pair[1].record()
        # dense tensors: Average -> compensate(accumulate=False) (dgc/compression.py:195-198,
        # 205-206), no ATen kernel: at W = 1 the Average is the identity and the wire cast a
        # rounding, fused into the compensate (dgc_compensate_wire, round_to fp16); at W > 1
        # the rank-order sum / W of the gathered rows, widened (dgc_compensate_ranks)
        if not self.exchanging:
            self._lib.check(L.dgc_compensate_wire(gd.data_ptr(), self._lib.VD[torch.float32], wt,
                                                  self.dense_mmt.data_ptr(), self.dense_out.data_ptr(),
                                                  self.n_dense, 0.9, int(self.nesterov), st), "dgc_compensate_wire")
            return
        if handle:
            src, stride = comm.synchronize(handle[0]).data_ptr(), self.dense_wire.numel()
        else:
            src, stride = b.gathered.data_ptr() + b.extra_off, b.rank_stride
        self._lib.check(L.dgc_compensate_ranks(ctypes.c_void_p(src), wt, comm.size(), stride,
                                               self.dense_mmt.data_ptr(), self.dense_out.data_ptr(), self.n_dense,
                                               0.9, int(self.nesterov), st), "dgc_compensate_ranks")

    def probe_buffers(self):
        b = self.b
        return [self.grads[0][0], self.grads[1][0], b.out_flat], [b._mmt_flat, b._vec_flat]

    def k1_bytes(self):
        # every compressed tensor: read g, mmt, vec; write mmt, vec; plus the samples written
        return 20 * self.n_comp + 4 * sum(a[1] + 1 for a in self.b.attrs if a[1] != 0)

    def records(self):
        return self.b.infos()

    def info(self):
        infos = self.b.infos()
        branches = {}
        for i in infos:
            branches[i["branch"]] = branches.get(i["branch"], 0) + 1
        return {"tensors": len(infos), "count": sum(i["count"] for i in infos), "branches": branches,
                "full_passes": sum(i["full_passes"] for i in infos),
                "exact_resamples": sum(i["tie_rule"] == "exact" for i in infos)}

    def config(self):
        return {"compressed_tensors": len(self.b.names), "compressed_elements": self.n_comp,
                "dense_elements": self.n_dense, "num_selects_total": self.b.capacity, "fill": self.b.fill,
                "exchange_parts": self.b.parts, "resample_order": self.b.resample_order}


class DropinRun:
    """A model's step through the drop-in API, as the reference's training loop drives it
    (dgc/horovod/optimizer.py:91-187, train.py:137-140): nn.Parameters of the model's
    shapes, DGCSGDMemory + DGCCompressor (initialised on the dim > 1 tensors), and
    dgc.horovod.DistributedOptimizer around a torch optimizer — ``batch`` True (one grouped
    step, dense zero_()), "sparse" (its re-zero of the previous entries) or False (the
    reference's per-tensor hooks: a compress with one host sync per tensor). One step =
    fresh p.grad tensors as backward hands them over (a distinct gradient set per step,
    the values of ModelRun's two sets), the grad-accumulator hooks fired in backward's
    (reverse) order, ``synchronize()`` (compress -> exchange -> decompress -> p.grad), and
    ``zero_grad()`` (set_to_none=True, torch's default). The wrapped optimizer's own update
    is not on the DGC path and is not run. W = 1 needs HOROVOD_ELASTIC=1 for the hooks
    (dgc/horovod/optimizer.py:79-80)."""

    def __init__(self, wl, rank, world, dev, batch, steps):
        import random
        from dgc import workloads
        from dgc.compression import DGCCompressor
        from dgc.horovod import DistributedOptimizer
        from dgc.memory import DGCSGDMemory
        os.environ.setdefault("HOROVOD_ELASTIC", "1")
        shapes = getattr(workloads, wl["model"])()
        comp_shapes, dense_shapes = workloads.split(shapes)
        self.named = [(n, torch.nn.Parameter(torch.zeros(s, device=dev))) for n, s in shapes]
        params = dict(self.named)
        compression = DGCCompressor(wl["ratio"], memory=DGCSGDMemory(momentum=0.9, nesterov=wl["nesterov"]),
                                    fp16_values=wl["fp16"], int32_indices=wl["int32"])
        with contextlib.redirect_stdout(io.StringIO()):
            compression.memory.initialize(self.named)
            compression.initialize([(n, params[n]) for n, _ in comp_shapes])
        random.seed(42)
        inner = torch.optim.SGD([p for _, p in self.named], lr=0.0)
        kw = {} if batch == "auto" else {"batch": batch}   # "auto": the drop-in default, no argument
        self.opt = DistributedOptimizer(inner, named_parameters=self.named, compression=compression, **kw)
        self.batched = self.opt._batched is not None
        # ModelRun's per-step gradient sets, value for value, as per-parameter tensors (the
        # per-tensor path decompresses into p.grad in place: a distinct set per step)
        gen = torch.Generator(device=dev)
        self.sets = []
        for s_ in range(steps):
            gen.manual_seed(gradient_seed(rank, s_))
            g = {n: torch.randn(workloads.numel(sh), generator=gen, device=dev).mul_(1e-3).view(sh)
                 for n, sh in comp_shapes}
            nd = sum(workloads.numel(sh) for _, sh in dense_shapes)
            d = torch.randn(nd, generator=gen, device=dev).mul_(1e-3)
            o = 0
            for n, sh in dense_shapes:
                g[n] = d[o: o + workloads.numel(sh)].clone().view(sh)
                o += workloads.numel(sh)
            self.sets.append([g[n] for n, _ in self.named])
        self.elements = sum(p.numel() for _, p in self.named)
        self.hooks = list(reversed(self.opt._hook_fns))

    def step(self, i, ev=None):
        for (_, p), g in zip(self.named, self.sets[i % len(self.sets)]):
            p.grad = g
        for _, hook in self.hooks:
            hook()
        self.opt.synchronize()
        self.opt.zero_grad()


def data_note(wl, run, nsteps, inputs="per-step"):
    per = ("a fresh gradient per rank and step, seed 0xD6C + 1000*rank + step (SURVEY.md §8d), generated in "
           "HBM before the timed region")
    if inputs == "alternating":
        per = ("--inputs alternating: 2 gradient buffers per rank (seeds 0xD6C + 1000*rank + {0, 1}), steps "
               "alternate between them (rounds 1-5's input model, not SURVEY.md §8d's)")
    elif "buffers" in wl:
        per = (f"{wl['buffers']} gradient buffers per rank (seeds 0xD6C + 1000*rank + {{0, 1}}), steps alternate "
               f"between them: a buffer per step would need {nsteps} x {4 * run.N / 1e9:.0f} GB of HBM")
    elif run.nbuf < nsteps:
        per += f" ({run.nbuf} buffers fit in HBM: steps cycle through them)"
    kind = {"normal": "N(0,1)", "bf16": "N(0,1) rounded to bf16 (held in fp32)"}.get(wl.get("grad"), "N(0,1) x1e-3")
    return (f"synthetic: torch.randn {kind} gradients, {per}; sample starts from random.Random(42); "
            "momentum/velocity state evolves across steps from zero")


def timed_steps(run, steps, warmup, world):
    """ms per step of ``run.step`` over ``steps`` steps after ``warmup`` (barrier +
    synchronize on both sides, max over ranks); step i takes gradient set i."""
    for i in range(warmup):
        run.step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        run.step(warmup + i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    return el * 1e3 / steps


def dropin_compare(model, rank, world, dev, steps, warmup):
    """The drop-in training step against the engine it wraps, same box, same gradients:
    DGCBatch alone (ModelRun, both fills), DistributedOptimizer with no batch argument
    (its default, "auto": the batched step here), batch="sparse", and the reference's
    per-tensor hook path (batch=False; few steps: it syncs per tensor)."""
    wl = dict(WORKLOADS[model])
    res = {"model": model, "steps": steps, "warmup": warmup}
    for fill in ("inline", "sparse"):
        run = ModelRun(wl, rank, world, dev, fill, steps + warmup)
        res[f"dgcbatch_{fill}_ms"] = round(timed_steps(run, steps, warmup, world), 4)
        del run
    for label, batch, n in (("optimizer_default_ms", "auto", steps), ("optimizer_batch_sparse_ms", "sparse", steps),
                            ("optimizer_per_tensor_ms", False, max(3, steps // 4))):
        run = DropinRun(wl, rank, world, dev, batch, n + warmup)
        res[label] = round(timed_steps(run, n, warmup, world), 4)
        del run
        torch.cuda.empty_cache()
    res["default_vs_dgcbatch"] = round(res["optimizer_default_ms"] / res["dgcbatch_inline_ms"], 3)
    res["batch_sparse_vs_dgcbatch"] = round(res["optimizer_batch_sparse_ms"] / res["dgcbatch_sparse_ms"], 3)
    res["note"] = ("ms per step; dgcbatch = the engine alone (gradients planted in its flat buffer); optimizer = "
                   "dgc.horovod.DistributedOptimizer: fresh p.grad tensors, hooks in backward order, synchronize(), "
                   "zero_grad(set_to_none=True); inline = the reference's dense zero_(), sparse = re-zero of the "
                   "previous entries")
    return res


CEILING_BYTES = 256 << 20   # per rank: the large-message allgather that bounds what RCCL can give here


def allgather_probe(run, world, reps=5):
    """The step's exchange alone, after the timed steps, with HIP events on the compute
    stream around issue + completion: one RCCL allgather of the packed payload issued
    both ways (``comm.COLLECTIVE_ISSUE``: on the current stream, async_op=False; on
    torch's collective stream, async_op=True + wait), the split exchange's parts when
    there are any, and a same-run ceiling — ``all_gather_into_tensor`` of 256 MB per rank
    (its bus bandwidth is the most RCCL moves over these links in this run)."""
    from dgc import comm
    b = run.b
    pay = b.payload
    dev = pay.device
    out = torch.empty(world * pay.numel(), dtype=torch.uint8, device=dev)

    def timed(fn, n=reps):
        fn()
        dist.barrier()
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return a.elapsed_time(e) / n

    res = {"single_ms": timed(lambda: dist.all_gather_into_tensor(out, pay, async_op=False)),
           "single_async_wait_ms": timed(lambda: dist.all_gather_into_tensor(out, pay, async_op=True).wait())}
    if getattr(b, "xchg", None) is not None:
        x = b.xchg
        g = torch.empty_like(x.gathers[0])

        def split():
            for h in x.send(pay, g):
                h.wait()
        res.update(parts=x.parts, split_ms=timed(split))
    big = torch.empty(CEILING_BYTES, dtype=torch.uint8, device=dev)
    big_out = torch.empty(world * CEILING_BYTES, dtype=torch.uint8, device=dev)
    res["ceiling_bytes_per_rank"] = CEILING_BYTES
    res["ceiling_ms"] = timed(lambda: dist.all_gather_into_tensor(big_out, big, async_op=False), 3)
    del big, big_out
    res["issue_default"] = comm.COLLECTIVE_ISSUE
    return res


def selection_steps(run, steps, start):
    """The selection records of ``steps`` more steps after the timed ones (untimed: each
    step's per-tensor records are read back, a host sync per step): branches over
    tensor-steps, full select passes per step, the resamples by tie rule, and how often
    the resample's multi-workgroup phases fell back — K5's global phase not co-resident
    (k5_fallback) or recovered after a barrier timeout (k5_recovered), K5s's set path not
    co-resident (k5s_fallback) or broken (k5s_broken): exact results either way, slower."""
    agg = {"steps": steps, "branches": {}, "full_passes_per_step": [], "resamples": {"set": 0, "exact": 0},
           "max_resample_candidates": 0, "k5_fallback": 0, "k5_recovered": 0, "k5s_fallback": 0, "k5s_broken": 0}
    for i in range(steps):
        run.step(start + i)
        recs = run.records()
        agg["full_passes_per_step"].append(sum(r["full_passes"] for r in recs))
        for r in recs:
            agg["branches"][r["branch"]] = agg["branches"].get(r["branch"], 0) + 1
            if r["branch"] == "resample":
                agg["resamples"][r["tie_rule"]] = agg["resamples"].get(r["tie_rule"], 0) + 1
                agg["max_resample_candidates"] = max(agg["max_resample_candidates"], r["candidates"])
            for key in ("k5_fallback", "k5_recovered", "k5s_fallback", "k5s_broken"):
                agg[key] += int(r[key])
    return agg


def hbm_probe(reads, writes, reps=5):
    """This box's streaming rate for K1's access mix, measured in the same run:
    dgc_hbm_probe (3 non-temporal 16-B reads + 2 writes per float4, one-shot blocks,
    K1's shape without its arithmetic) over the workload's own buffers after the timed
    steps, HIP events on the stream it runs on, best of ``reps``. MI355X boxes differ
    by ~10 % (the same library ran K1 in 3.29 and 3.68 ms on two boxes,
    tools/ab_k1.py), so K1 is also reported as a fraction of this."""
    from dgc import _lib
    L = _lib.lib()
    n = min(t.numel() for t in reads + writes)
    dev = reads[0].device
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(L.dgc_hbm_probe(*(t.data_ptr() for t in reads), *(t.data_ptr() for t in writes), n,
                                   _lib.stream_of(dev)), "dgc_hbm_probe")
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1)
        best = t if best is None else min(best, t)
    nbytes = 20 * (n // 4) * 4
    return {"kind": "dgc_hbm_probe: K1's access shape, 3 reads + 2 writes of 16 B per float4", "bytes": nbytes,
            "ms": best, "GBs": nbytes / (best * 1e-3) / 1e9}


def step_bytes(run, world, full_passes):
    """Bytes one rank must move per step (per compressed element):
    compensate 20 + select re-read 4 (0 when the K1 candidate lists serve the
    selection) + dense decompress write 4, the samples 4S, masking 8k, payload written
    k(vb+ib) + gathered W*k(vb+ib) read, scatter RMW 8Wk. `contract` keeps the 28 B
    of SURVEY.md §8d; `required` is what this step's path actually needs: no re-read
    when the lists serve, and for a persistent output (fill "sparse": bucket or batch)
    a re-zero of the previous step's W*k slots (4 B each) instead of the dense 4 B/elem."""
    n = run.n_comp if isinstance(run, ModelRun) else run.N
    k, S = run.k, run.S
    sparse = 4 * S + 8 * k + (1 + world) * k * (run.vbytes + run.ibytes) + 8 * world * k
    contract = 28 * n + sparse
    rezero = run.b.fill == "sparse"
    required = (20 + (0 if full_passes == 0 else 4) + (0 if rezero else 4)) * n + sparse + (4 * world * k if rezero else 0)
    if isinstance(run, ModelRun):   # dense tensors: read g, mmt; write mmt, out
        contract += 16 * run.n_dense
        required += 16 * run.n_dense
    return contract, required


@contextlib.contextmanager
def _stdout_to_stderr():
    """File-descriptor level: RCCL prints its version banner to stdout when a
    communicator comes up; the bench's stdout carries the one JSON line only."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _init_group(dev, **kw):
    with _stdout_to_stderr():
        dist.init_process_group("nccl", device_id=dev, **kw)
        dist.barrier()   # the communicator is up (and has printed) before stdout is back


# ---------------------------------------------------------------------------- main
def main():
    args = parse()
    check_devices(args.gpus, torch.cuda.device_count())
    envs = launch_plan(args.gpus, os.environ)
    if envs is not None:
        sys.exit(spawn(envs))
    wl = WORKLOADS[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = None
    one_rank = args.rccl_one_rank and world == 1
    if world > 1:
        _init_group(dev)
        backend = dist.get_backend()
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} but the process group has {dist.get_world_size()} ranks")
    elif one_rank:   # a one-rank RCCL group, the engines exchanging through it (dgc/comm.py)
        from dgc import comm
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        _init_group(dev, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        comm.ONE_RANK_SHORTCUT = False
        backend = dist.get_backend()
    coll = world > 1 or one_rank
    nsteps = args.warmup + args.steps
    nbufs = 2 if args.inputs == "alternating" else nsteps
    run = (FlatRun(wl, rank, world, dev, args.fill, nbufs) if wl["kind"] == "flat" else
           ModelRun(wl, rank, world, dev, args.fill, nbufs))

    log(f"{args.workload}: rank {rank}/{world} set up")
    phases = ("compensate", "select", "allgather", "decompress")
    for i in range(args.warmup):
        run.step(i)
    torch.cuda.synchronize()
    # HIP events in the timed steps: K1 (the roofline kernel) always; the allgather when
    # there is one (its bus bandwidth); every phase only with --phases — each event pair
    # costs the GPU a few µs of idle time, ~7 % of a ResNet-50 step with all four phases
    timed = phases if args.phases else (("compensate", "allgather") if coll else ("compensate",))
    evs = [{p: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for p in timed}
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    # the collectives the timed steps issue (counted on the host: each is one Python call)
    counts = {"all_gather_into_tensor": 0, "all_reduce": 0}
    saved = {name: getattr(dist, name) for name in counts}
    if coll:
        def counted(name):
            fn = saved[name]

            def wrapper(*a, **kw):
                counts[name] += 1
                return fn(*a, **kw)
            return wrapper
        for name in counts:
            setattr(dist, name, counted(name))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run.step(args.warmup + i, evs[i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    for name, fn in saved.items():
        setattr(dist, name, fn)
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = {p: sum(e[p][0].elapsed_time(e[p][1]) for e in evs) / args.steps for p in timed}
    info = run.info()
    extras = {}
    if coll and not args.no_extras and getattr(run.b, "xchg", None) is None:
        # the step again with the single allgather issued the other way (dgc/comm.py
        # COLLECTIVE_ISSUE): on the current stream vs on torch's collective stream + wait
        from dgc import comm
        mode = comm.COLLECTIVE_ISSUE
        other = "async" if mode == "current" else "current"
        comm.COLLECTIVE_ISSUE = other
        try:
            other_ms = timed_steps(run, args.steps, 2, world)
        finally:
            comm.COLLECTIVE_ISSUE = mode
        extras["issue_modes"] = {
            "default": mode, f"{mode}_ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            f"{other}_ms_per_step": round(other_ms, 4),
            "note": "current = all_gather_into_tensor(async_op=False), run by torch on the caller's stream; async = "
                    "async_op=True + wait(), on torch's collective stream joined by events"}
    if not args.no_extras and run.b.fill == "sparse":
        # the same steps with the reference's dense zero_() (dgc/compression.py:191) before
        # the scatter: what the persistent output's re-zero saves. The flat bucket goes on
        # from the same state; a model set gets a fresh batch built with fill="inline"
        # (its step count and gradients as above)
        if wl["kind"] == "flat":
            run.b.fill = "inline"
            dense = timed_steps(run, args.steps, 2, world)
            run.b.fill = "sparse"
        else:
            dense = timed_steps(ModelRun(wl, rank, world, dev, "inline", nbufs), args.steps, args.warmup, world)
        extras["dense_fill"] = {"ms_per_step": round(dense, 4), "steps": args.steps,
                                "note": "fill inline: the whole output zeroed every step (4 B/elem), as the "
                                        "reference's grad.zero_(); value/ms_per_step above use fill sparse"}
    xgmi = allgather_probe(run, world) if coll else None
    sel_steps = selection_steps(run, args.steps, nsteps)
    probe = hbm_probe(*run.probe_buffers())   # after the timed steps: overwrites the state
    ms_step = elapsed * 1e3 / args.steps
    full_passes = info.get("full_passes", 0)
    contract, required = step_bytes(run, world, full_passes)
    k1_bytes = run.k1_bytes()
    traffic, traffic_src = pmc_traffic(args.workload)
    prof_ms, prof_src = rocprof_k1_ms(args.workload)
    if rank != 0:
        if coll:
            dist.destroy_process_group()
        return
    k1_ms = ms["compensate"]   # HIP events around K1's launch on the stream it runs on
    if wl["kind"] == "flat":
        k1_name = "K1 compensate + fused sample + speculative lists (k_compensate_list)"
    else:
        k1_name = "K1 over all compressed tensors (k_compensate_list, one launch)"
    k1_gbs = k1_bytes / (k1_ms * 1e-3) / 1e9
    wire = f"{'fp16' if run.vbytes == 2 else 'fp32'} values / {'int32' if run.ibytes == 4 else 'int64'} indices"
    res = {
        "metric": METRIC,
        "value": world * run.elements / (ms_step * 1e-3),
        "unit": "grad elements/s",
        "n_gpus": world,
        "world_size": dist.get_world_size() if world > 1 else 1,
        "backend": ((f"{backend} (RCCL over xGMI)" if backend == "nccl" else backend) if world > 1 else
                    "nccl (RCCL, one rank: --rccl-one-rank)" if one_rank else "none (1 rank)"),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "vs_baseline_note": "null: BASELINE.md holds no published number for this metric (the reference publishes "
                            "none); the CPU restatement of the reference timed on this host is cpu_baseline",
        "dtype": "f32",
        "data": data_note(wl, run, nsteps, args.inputs),
        "config": dict({"workload": f"{args.workload} ({wl['config']})", "compress_ratio": wl["ratio"],
                        "nesterov": wl["nesterov"], "momentum": 0.9, "momentum_masking": True, "wire": wire,
                        "parallelism": f"dp{world}", "inputs": args.inputs}, **run.config()),
        "roofline": {"kernel": k1_name, "bound": "hbm", "achieved": k1_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": k1_gbs / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": k1_bytes, "avg_launch_ms": k1_ms,
                     "rocprof_avg_launch_ms": prof_ms, "rocprof_source": prof_src},
        "step_hbm": {"required_bytes_per_rank": required, "contract_bytes_per_rank": contract,
                     "achieved_GBs": required / (ms_step * 1e-3) / 1e9,
                     "frac_of_8TBs": required / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "frac_of_measured_copy": required / (ms_step * 1e-3) / 1e9 / HBM_COPY_GBS},
        "hbm_probe": dict(probe, k1_frac_of_probe=k1_gbs / probe["GBs"],
                          step_frac_of_probe=required / (ms_step * 1e-3) / 1e9 / probe["GBs"]),
        "phase_ms": {p: round(v, 4) for p, v in ms.items()},
        "compensate_ms_per_step": [round(e["compensate"][0].elapsed_time(e["compensate"][1]), 3) for e in evs],
        "selection": info,
        "selection_steps": sel_steps,
    }
    if coll:
        res["collectives_per_step"] = {name: c / args.steps for name, c in counts.items()}
    if xgmi is not None and world == 1:   # --rccl-one-rank: the collective's own cost, no link traffic
        res["allgather"] = dict({"payload_bytes_per_rank": run.payload,
                                 "note": "one rank: the RCCL collectives' cost without link traffic (ceiling_ms: "
                                         "a 256 MB one-rank allgather, i.e. a device copy)"}, **xgmi)
    elif xgmi is not None:
        bus = (world - 1) * run.payload / (xgmi["single_ms"] * 1e-3) / 1e9
        ceiling = (world - 1) * xgmi["ceiling_bytes_per_rank"] / (xgmi["ceiling_ms"] * 1e-3) / 1e9
        res["allgather"] = dict({"payload_bytes_per_rank": run.payload, "bus_GBs": bus,
                                 "peak_GBs": (world - 1) * XGMI_LINK_GBS, "frac": bus / ((world - 1) * XGMI_LINK_GBS),
                                 "ceiling_GBs": ceiling, "frac_of_ceiling": bus / ceiling,
                                 "ceiling_frac_of_links": ceiling / ((world - 1) * XGMI_LINK_GBS),
                                 "note": "bus GB/s = (W-1) x bytes per rank / time; one all_gather_into_tensor of the "
                                         "packed payload alone after the timed steps (HIP events on the compute "
                                         "stream around issue + completion); peak = (W-1) x 153 GB/s of xGMI links; "
                                         "ceiling = the same collective of 256 MB per rank in this run"}, **xgmi)
    log(f"{args.workload}: {ms_step:.3f} ms/step on the GPU")
    if world == 1 and not args.no_extras:
        model = wl["model"] if wl["kind"] == "model" else args.dropin_model
        try:
            log(f"drop-in DistributedOptimizer comparison on {model}")
            res["dropin"] = dropin_compare(model, rank, world, dev, 20, 5)
        except Exception as e:   # an extra must not cost the headline line
            res["dropin"] = {"error": f"{type(e).__name__}: {e}"}
    res.update(extras)
    if world == 1 and not args.no_cpu:
        cores = cpu_cores()
        log(f"CPU baseline on {cores} threads, then 1 thread")
        res["cpu_baseline"] = cpu_baseline(run, wl, args.cpu_numel, args.cpu_steps, cores)
        res["cpu_baseline_1thread"] = cpu_baseline(run, wl, args.cpu_numel_1t, 2, 1)
    print(json.dumps(res), flush=True)
    if coll:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
