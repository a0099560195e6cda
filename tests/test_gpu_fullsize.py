"""Parity at the bench's own size: the 1e9-element flat bucket (BASELINE configs[3])
stepped through dgc.bucket.DGCBucket exactly as bench.py steps it (the same two
alternating seeded gradients, ratio 0.001, nesterov), compared with the numpy oracle
after EVERY step: the transmitted indices (in order) and values, momentum and
velocity, and the decompressed dense gradient, all bit for bit. The steady state the
bench times — K1's speculative candidate lists serving the selection, spilled lists,
the trunc branch — is reached and recorded."""
import random
import sys

import numpy as np
import pytest
import torch

from oracle import dgc_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
CH = 1 << 27   # host comparisons in 512 MB chunks


def _equal_bits(gpu, host):
    n = host.size
    for c0 in range(0, n, CH):
        c1 = min(n, c0 + CH)
        if not np.array_equal(gpu[c0:c1].cpu().numpy().view(np.uint32), host[c0:c1].view(np.uint32)):
            return False
    return True


@pytest.mark.timeout(1200)
def test_flat_1b_bucket_steps_match_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    free, _ = torch.cuda.mem_get_info()
    if free < 40 * 2 ** 30:
        pytest.skip("needs ~40 GiB of free HBM")
    from dgc.bucket import DGCBucket
    N, steps = 10 ** 9, 10
    b = DGCBucket(N, compress_ratio=1e-3, momentum=0.9, nesterov=True, device=DEV, seed=42)
    attrs = O.attributes(N, 1e-3)
    rng = random.Random(42)
    gen = torch.Generator(device=DEV)
    grads = []
    for s in range(2):   # bench.py's FlatRun: seeds 0xD6C + 1000*rank + buffer, rank 0
        gen.manual_seed(0xD6C + s)
        grads.append(torch.randn(N, generator=gen, device=DEV))
    out = torch.empty(N, device=DEV)
    m_o = np.zeros(N, np.float32)
    v_o = np.zeros(N, np.float32)
    seen = []
    for s in range(steps):
        g = grads[s % 2]
        start = rng.randint(0, attrs[4] - 1)
        b.step(g, out)
        torch.cuda.synchronize()
        info = b.last_info()
        ov, oi, oinfo = O.compress_step(g.cpu().numpy(), m_o, v_o, attrs, start, nesterov=True)
        n = info["count"]
        gi = b.payload[b.ioff: b.ioff + 8 * n].view(torch.int64).cpu().numpy()
        gv = b.payload[b.voff: b.voff + 4 * n].view(torch.float32).cpu().numpy()
        assert info["branch"] == oinfo["branch"], (s, info)
        assert np.array_equal(gi, oi), (s, info)
        assert np.array_equal(gv.view(np.uint32), ov.view(np.uint32)), s
        if s % 3 == 2 or s == steps - 1:   # reading flushes the deferred masking: most steps leave it to K1
            assert _equal_bits(b.vec, v_o) and _equal_bits(b.mmt, m_o), s
        dense = np.zeros(N, np.float32)
        dense[oi] = ov    # W = 1: unique indices, scale 1
        assert _equal_bits(out, dense), s
        del dense
        seen.append((info["branch"], info["full_passes"], info["overflow_segments"]))
        print(f"step {s}: {info}", file=sys.stderr, flush=True)
    # the bench's steady state was exercised: selections served by the K1 lists
    assert any(fp == 0 for _, fp, _ in seen[1:]), seen
