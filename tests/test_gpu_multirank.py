"""The product path at world size 2 on one MI355X: two processes on cuda:0 over gloo
(dgc.comm stages the exchange through the host), everything else the HIP path —
compress (K1/K3/K4/K5), the packed allgather, synchronize, the packed decompress with
its regrouping of topk-ordered runs, DGCSGD's fused step.

* The reference's DistributedOptimizer runs (optimizer.npz: 3 steps; ResNet-20 =
  BASELINE configs[0]: 6 steps over the 0.316 -> 0.1 -> 0.001 warmup with
  re-initialisation, fp16 values / int32 indices) are replayed from the recorded
  per-step gradients and hook order; the weights must equal the reference's bit for
  bit — per tensor as the reference runs, and with batch=True (one grouped K1 /
  allgather / decompress and one dense allreduce per step).
* DGCBucket at W=2, every fill mode, against the oracle over both ranks' payloads.
"""
import pytest
import torch
import torch.multiprocessing as mp

import dist_helpers as H
import gpu_dist_helpers as G

pytestmark = pytest.mark.gpu


def run(fn, world, *args):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = H.free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=150)
        if p.exitcode is None:
            p.kill()
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    out = {}
    while not q.empty():
        rank, res = q.get()
        out[rank] = res
    assert sorted(out) == list(range(world))
    return out


@pytest.mark.timeout(200)
@pytest.mark.parametrize("batch", [False, True, "default"], ids=["per-tensor", "batched", "default"])
@pytest.mark.parametrize("label", ["tinynet", "resnet20"])
def test_distributed_optimizer_w2_reproduces_reference_weights(label, batch):
    out = run(G.optimizer_replay_worker, 2, label, batch)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("batch", [False, True, "default"], ids=["per-tensor", "batched", "default"])
@pytest.mark.parametrize("label,mode,resume_at", [("resnet20", "fresh", 2), ("resnet20", "fresh", 4),
                                                  ("resnet20", "inplace", 4), ("tinynet", "inplace", 1)])
def test_checkpoint_resume_w2_reproduces_reference_weights(label, mode, resume_at, batch):
    """train.py's checkpoint (model, optimizer, compression.memory state dicts) at an
    epoch boundary and a resume — into fresh objects, or into the running ones after
    the state moved on — continue exactly as the uninterrupted reference run: the weights
    after every later step equal the goldens, per tensor and batched (whose flat layout
    must take the loaded memory tensors back in, and whose deferred masking must be
    flushed into the checkpoint)."""
    out = run(G.resume_worker, 2, label, batch, mode, resume_at)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("fill,kind", [("inline", "normal"), ("allgather", "normal"), ("allgather", "layered"),
                                       ("sparse", "normal"), ("sparse", "layered")])
def test_bucket_w2_matches_oracle(fill, kind):
    out = run(G.bucket_worker, 2, fill, kind)
    for rank, res in out.items():
        problems = [r for r in res if r[0] != "branches"]
        assert problems == [], (rank, res)
    if kind == "layered":
        assert "resample" in dict(out[0])["branches"]


@pytest.mark.parametrize("world,fill,kind", [(2, "sparse", "normal"), (2, "sparse", "layered"),
                                              (2, "inline", "normal"), (4, "sparse", "normal")])
def test_batch_multirank_matches_oracle(world, fill, kind):
    """DGCBatch with W ranks (processes) on one MI355X: one payload of every tensor,
    one allgather, the decompress into the batch's persistent output (fill "sparse":
    the previous step's W runs re-zeroed), against the oracle per tensor."""
    out = run(G.batch_worker, world, fill, kind)
    for rank, res in out.items():
        problems = [r for r in res if r[0] != "branches"]
        assert problems == [], (rank, res)


@pytest.mark.timeout(240)
@pytest.mark.parametrize("fill", ["allgather", "sparse"])
def test_bucket_w4_matches_oracle(fill):
    """4 ranks (processes) on one MI355X: the 4-run decompress (bounds + wave scatter +
    crowded-chunk path) with the side-stream zero fill under the exchange or the sparse
    re-zero of the persistent output, against the oracle over all four ranks' payloads."""
    out = run(G.bucket_worker, 4, fill, "normal")
    for rank, res in out.items():
        problems = [r for r in res if r[0] != "branches"]
        assert problems == [], (rank, res)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,parts,fill,kind", [(2, 2, "inline", "normal"), (2, 3, "sparse", "layered"),
                                                   (4, 2, "allgather", "normal"), (4, 4, "sparse", "normal"),
                                                   (8, 4, "sparse", "normal"), (8, 8, "inline", "layered")])
def test_bucket_split_exchange_matches_oracle(world, parts, fill, kind):
    """The allgather in `parts` collectives, each part scattered as it lands
    (dgc/exchange.py), at W = 2 / 4 / 8 ranks on one MI355X over gloo: every fill form,
    against the oracle over all ranks' payloads, step by step."""
    out = run(G.bucket_worker, world, fill, kind, parts)
    for rank, res in out.items():
        problems = [r for r in res if r[0] != "branches"]
        assert problems == [], (rank, res)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,parts,fill,kind", [(2, 2, "sparse", "layered"), (4, 2, "inline", "normal"),
                                                   (8, 4, "sparse", "normal")])
def test_batch_split_exchange_matches_oracle(world, parts, fill, kind):
    out = run(G.batch_worker, world, fill, kind, parts)
    for rank, res in out.items():
        problems = [r for r in res if r[0] != "branches"]
        assert problems == [], (rank, res)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("case", ["fp16_w2_fp16v_i32"])
def test_half_w2_communicate_matches_reference(case):
    """bf16 / fp16 parameters through the real exchange (compress -> communicate ->
    synchronize -> decompress, gloo) at the golden case's world size: payloads, 16-bit
    velocity and decompressed gradient equal the reference's (tests/golden/half.*)."""
    out = run(G.half_worker, 2, case)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("fp16", [False, True], ids=["wire-dtype", "wire-fp16"])
@pytest.mark.parametrize("dtype", ["bfloat16", "float16"])
def test_half_batched_optimizer_w2_equals_per_tensor(dtype, fp16):
    """bf16 / fp16 parameters through DistributedOptimizer(batch=True) at W = 2 (two
    processes on one MI355X over gloo): the per-tensor path's gradients and 16-bit state
    (that path is pinned to the reference's 16-bit fixtures) bit for bit, 4 steps."""
    out = run(G.half_batch_worker, 2, dtype, fp16)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("batch", [False, True], ids=["per-tensor", "batched"])
@pytest.mark.parametrize("label", ["w3_fp32", "w3_fp16", "w4_fp16", "w8_fp32", "w8_fp16", "w4_fp16_wm5o"])
def test_distributed_optimizer_dense_average_reproduces_reference_weights(label, batch):
    """The dense tensors' Average at W = 3 / 4 / 8 (tests/golden/optimizer_multi.*, the
    reference's DistributedOptimizer + DGCSGD on TinyNet; fp32 and fp16 wire values; a
    wm5o run whose first epoch sends every tensor dense): the rank-order sum in the wire
    dtype, then / W (dgc/compression.py:205-206 as the oracle restates Horovod's
    Average) — per tensor through dgc.comm's allgather + dgc_rank_sum, batched in the
    tail of the one packed payload. Weights bit for bit after every step, every rank."""
    import json
    import os
    W = json.load(open(os.path.join(G.GOLDEN, "optimizer_multi.json")))[label]["W"]
    out = run(G.multi_replay_worker, W, label, batch)
    for rank, problems in out.items():
        assert problems == [], (rank, problems)
