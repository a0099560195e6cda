"""Cost of the flat bucket's selection when the speculative lists MISS (every other
step the gradient scale drops 20x, so the sampled threshold falls below the list
threshold and the full passes run): ms per step over a few steps, for comparing the
chained launch (k_chain_one) with the separate launches (DGC_NO_CHAIN=1).

  python tools/chain_probe.py [numel] [steps]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "adam-compression_amd")]

import torch  # noqa: E402


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1e9
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    from dgc.bucket import DGCBucket
    dev = torch.device("cuda:0")
    b = DGCBucket(n, compress_ratio=0.001, momentum=0.9, nesterov=True, device=dev, seed=42)
    g = torch.randn(n, device=dev)
    out = torch.empty(n, device=dev)
    scales = [1.0, 0.05]
    for s in range(4):   # warm-up
        b.step(g * scales[s % 2], out)
    torch.cuda.synchronize()
    grads = [g * sc for sc in scales]
    t = []
    for s in range(steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.step(grads[s % 2], out)
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) * 1e3)
        info = b.last_info()
        print(f"step {s}: {t[-1]:.3f} ms branch {info['branch']} full_passes {info['full_passes']} "
              f"recounts {info['recounts']}", flush=True)
    print(f"mean {sum(t) / len(t):.3f} ms  (DGC_NO_CHAIN={os.environ.get('DGC_NO_CHAIN', '')})")


if __name__ == "__main__":
    main()
