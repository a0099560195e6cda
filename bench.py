#!/usr/bin/env python3
"""DGC hot-path benchmark on MI355X: one flat fp32 gradient bucket per rank through
compensate -> compress (sample, threshold, select, masking) -> RCCL allgather ->
decompress, all on the device (BASELINE.json configs[3]: 1B elements, ratio 0.001,
nesterov, momentum 0.9, fp32/int64 wire; 1/2/4/8 GPUs, weak scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--numel 1e9] [--no-cpu]
    torchrun --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line. ``value`` = grad elements processed by all ranks per
second (each rank compresses its own N-element gradient). ``roofline`` is for the
dominant kernel, K1 (compensate + fused sample), timed with HIP events on the
stream it runs on; the whole step's algorithmic HBM rate is reported beside it.
"""
import argparse
import json
import os
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--numel", type=float, default=1e9)
    ap.add_argument("--ratio", type=float, default=0.001)
    ap.add_argument("--cpu-numel", type=float, default=1e9, help="CPU-baseline sample size")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--phases", action="store_true", help="HIP events around every phase (adds markers)")
    return ap.parse_args()


def cpu_baseline(numel, ratio, steps):
    """The reference op sequence restated on torch CPU (oracle/torch_cpu.py), timed on
    this host's cores over a bounded sample of the workload (rank 0, N=1 only)."""
    from oracle import torch_cpu
    threads = torch.get_num_threads()
    N = int(numel)
    attrs = torch_cpu.attributes(N, ratio)
    g = torch.randn(N, generator=torch.Generator().manual_seed(1))
    mmt, vec, out = torch.zeros(N), torch.zeros(N), torch.empty(N)
    import random
    rng = random.Random(42)
    torch_cpu.cpu_step(g, mmt, vec, out, attrs, rng.randint(0, attrs[4] - 1))   # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        torch_cpu.cpu_step(g, mmt, vec, out, attrs, rng.randint(0, attrs[4] - 1))
    dt = (time.perf_counter() - t0) / steps
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": N / dt, "unit": "grad elements/s", "cores": threads, "kind": "port",
            "sample": f"{N} elements x {steps} steps (compensate+sparsify+update+decompress, W=1, "
                      f"torch {torch.__version__} CPU ops as the reference issues them), "
                      f"{dt * 1e3:.1f} ms/step on {threads} threads; {model}"}


def pmc_traffic(kernel_key="k_compensate_list"):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC profile
    of this bench (tools/gpu_check.sh: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
    passes; FETCH_SIZE x2 for gfx950's half count of wide reads, KB x 1024)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "round*", "pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    for k, v in d.items():
        if kernel_key in k:
            return v["hbm_bytes_per_launch_corrected"], os.path.relpath(files[-1], REPO)
    return None, None


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


def spawn(envs):
    """One child process per rank (started before this process touches the GPU);
    returns the first non-zero exit code, or 0."""
    import subprocess
    procs = [subprocess.Popen([sys.executable] + sys.argv, env=e) for e in envs]
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c != 0), 0)


def main():
    args = parse()
    envs = launch_plan(args.gpus, os.environ)
    if envs is not None:
        sys.exit(spawn(envs))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from dgc.bucket import DGCBucket, algorithmic_bytes

    N = int(args.numel)
    bucket = DGCBucket(N, compress_ratio=args.ratio, momentum=0.9, nesterov=True, device=dev, world_size=world)
    gen = torch.Generator(device=dev)
    grads = []
    for s in range(2):
        gen.manual_seed(0xD6C + 1000 * rank + s)
        grads.append(torch.randn(N, generator=gen, device=dev))
    out = torch.empty(N, device=dev)

    phases = ("compensate", "select", "allgather", "decompress")
    for i in range(args.warmup):
        bucket.step(grads[i % 2], out)
    torch.cuda.synchronize()
    timed = phases if args.phases else ("compensate", "allgather")
    evs = [{p: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for p in timed}
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        bucket.step(grads[i % 2], out, evs[i])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms = {p: sum(e[p][0].elapsed_time(e[p][1]) for e in evs) / args.steps for p in timed}
    info = bucket.last_info()
    ms_step = elapsed * 1e3 / args.steps
    k, S = bucket.k, bucket.num_samples
    step_bytes = algorithmic_bytes(N, k, S, world)
    k1_bytes = 20 * N + 4 * bucket.cnt            # read g, mmt, vec; write mmt, vec; write samples
    k1_gbs = k1_bytes / (ms["compensate"] * 1e-3) / 1e9
    payload = bucket.rank_stride
    traffic, traffic_src = pmc_traffic()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    res = {
        "metric": METRIC,
        "value": world * N / (ms_step * 1e-3),
        "unit": "grad elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: torch.randn N(0,1) fp32 gradients, 2 alternating buffers per rank "
                "(seed 0xD6C + 1000*rank + buffer); momentum/velocity state evolves across steps",
        "config": {"workload": "flat-1B-bucket (BASELINE configs[3])" if N == 10 ** 9 else f"flat-{N}-bucket",
                   "numel": N, "compress_ratio": args.ratio, "num_selects": k, "num_samples": S,
                   "sample_stride": bucket.stride, "nesterov": True, "momentum": 0.9, "momentum_masking": True,
                   "wire": "fp32 values / int64 indices", "parallelism": f"dp{world}"},
        "roofline": {"kernel": "K1 compensate + fused sample + speculative lists (k_compensate_list)",
                     "bound": "hbm",
                     "achieved": k1_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": k1_gbs / HBM_PEAK_GBS,
                     "traffic": traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": k1_bytes,
                     "avg_launch_ms": ms["compensate"]},
        "step_hbm": {"algorithmic_bytes_per_rank": step_bytes,
                     "achieved_GBs": step_bytes / (ms_step * 1e-3) / 1e9,
                     "frac_of_8TBs": step_bytes / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "frac_of_measured_copy": step_bytes / (ms_step * 1e-3) / 1e9 / HBM_COPY_GBS},
        "phase_ms": {p: round(v, 4) for p, v in ms.items()},
        "selection": info,
    }
    if world > 1 and ms["allgather"] > 0:
        bus = (world - 1) * payload / (ms["allgather"] * 1e-3) / 1e9
        res["allgather"] = {"payload_bytes_per_rank": payload, "bus_GBs": bus,
                            "peak_GBs": (world - 1) * XGMI_LINK_GBS,
                            "frac": bus / ((world - 1) * XGMI_LINK_GBS)}
    if world == 1 and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline(args.cpu_numel, args.ratio, args.cpu_steps)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
