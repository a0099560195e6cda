"""A/B of the flat-bucket step on one box: `python tools/ab_k1.py LIB.so [LIB2.so ...]`
runs the bench's flat-1B loop (20 timed steps after 5 warm-up) against each library
in a child process, alternating twice, and prints K1 / step times per library.
Symbols a library does not export are dropped from the ctypes table (older builds)."""
import ctypes
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    os.environ["DGC_HIP_LIB"] = lib
    sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]
    import torch
    from dgc import _lib
    h = ctypes.CDLL(lib)
    for name in list(_lib._SIGNATURES):
        if not hasattr(h, name):
            del _lib._SIGNATURES[name]
    from dgc.bucket import DGCBucket
    dev = torch.device("cuda:0")
    N = 10 ** 9
    b = DGCBucket(N, compress_ratio=1e-3, momentum=0.9, nesterov=True, device=dev, world_size=1)
    gen = torch.Generator(device=dev)
    grads = []
    for s in range(2):
        gen.manual_seed(0xD6C + s)
        grads.append(torch.randn(N, generator=gen, device=dev))
    out = torch.empty(N, device=dev)
    for i in range(5):
        b.step(grads[i % 2], out)
    torch.cuda.synchronize()
    ev = [{"compensate": (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))}
          for _ in range(20)]
    t0 = time.perf_counter()
    for i in range(20):
        b.step(grads[i % 2], out, ev[i])
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / 20 * 1e3
    k1 = sum(e["compensate"][0].elapsed_time(e["compensate"][1]) for e in ev) / 20
    print(json.dumps({"lib": lib, "step_ms": round(step, 4), "k1_ms": round(k1, 4)}), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    libs = sys.argv[1:]
    for _ in range(2):
        for lib in libs:
            subprocess.check_call([sys.executable, __file__, "--child", lib])


if __name__ == "__main__":
    main()
