"""Helpers for the multi-process CPU (gloo) tests.

``OracleDGCCompressor`` / ``OracleMemory`` are TEST DOUBLES: the product
``DGCCompressor`` runs only on the MI355X, so on CPU the compress / decompress
arithmetic is swapped for the numpy oracle while everything else — the drop-in
``DistributedOptimizer`` hooks, ``communicate`` / ``synchronize`` with the packed
payload, ``dgc.comm`` over torch.distributed — is the product code under test.
"""
import os
import random
import socket
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (REPO, os.path.join(REPO, "adam-compression_amd"), HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from dgc.compression import DGCCompressor, _Gathered  # noqa: E402
from dgc.comm import Average  # noqa: E402
from dgc.memory import DGCSGDMemory  # noqa: E402
from oracle import dgc_oracle as O  # noqa: E402
from models import ResNet20, TinyNet  # noqa: E402


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class OracleMemory(DGCSGDMemory):
    def compensate(self, grad, name, accumulate=True):
        g = grad.detach().reshape(-1).numpy()
        mmt = self.momentums[name].view(-1).numpy()
        if accumulate:
            vec = self.velocities[name].view(-1).numpy()
            O.compensate(g, mmt, vec, self.momentum, self.nesterov, True)
            return self.velocities[name]
        out = O.compensate(g, mmt, None, self.momentum, self.nesterov, False)
        return torch.from_numpy(out).view_as(self.momentums[name])

    def update(self, name, ctx):
        O.update(self.momentums[name].view(-1).numpy(), self.velocities[name].view(-1).numpy(),
                 ctx[0].reshape(-1).numpy().astype(np.int64), self.momentum_masking)


class OracleDGCCompressor(DGCCompressor):
    def compress(self, tensor, name):
        if self.compress_ratio < 1.0 and name in self.attributes:
            numel, shape, k, S, ks, stride = self.attributes[name]
            self.memory.compensate(tensor, name, accumulate=True)
            start = self._sample_start(name)
            vec = self.memory.velocities[name].view(-1).numpy()
            values, indices, _ = O.sparsify(vec, (numel, k, S, ks, stride), start,
                                            upper=self.compress_upper_bound, lower=self.compress_lower_bound,
                                            max_iters=self.max_adaptation_iters, resample=self.resample)
            self.memory.update(name, (torch.from_numpy(indices),))
            values, indices = O.wire_cast(values, indices, self.fp16_values, self.int32_indices)
            payload, lay = self._new_payload(name, tensor.device)
            n = values.size
            payload[:8].view(torch.int64).fill_(n)
            v, i = self._views(payload, lay, n)
            v.copy_(torch.from_numpy(values).view(-1, 1))
            i.copy_(torch.from_numpy(indices).view(-1, 1))
            self._payloads[name] = (payload, lay)
            return (v, i), (name, numel, shape, torch.float32, torch.int64, tensor.data.view(numel))
        return super().compress(tensor, name)

    def decompress(self, tensor, ctx):
        name, numel, shape, vdtype, idtype, grad = ctx
        if self.compress_ratio < 1.0 and name in self.attributes:
            values, indices = tensor
            assert isinstance(tensor, _Gathered) and tensor.run_offsets is not None
            W = len(tensor.run_offsets) - 1
            dense = O.decompress([values.reshape(-1).numpy()], [indices.reshape(-1).numpy()], numel,
                                 W, average=self.op == Average)
            grad.copy_(torch.from_numpy(dense))
            return grad.view(shape)
        if self.fp16_values and vdtype.is_floating_point:
            tensor = tensor.type(vdtype)
        return self.memory.compensate(tensor, name, accumulate=False)


def optimizer_worker(rank, world, port, golden_path, queue):
    """One rank of the reference's DistributedOptimizer + DGCSGD + DGC training loop,
    checked step by step against the weights the reference produced."""
    import contextlib
    import io

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgc.horovod import DistributedOptimizer
        from dgc.optim import DGCSGD
        golden = np.load(golden_path)
        torch.manual_seed(7)
        model = TinyNet()
        opt = DGCSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
        mem = OracleMemory(momentum=0.9)
        with contextlib.redirect_stdout(io.StringIO()):
            comp = OracleDGCCompressor(0.01, memory=mem)
            mem.initialize(model.named_parameters())
            comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        dopt = DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                    backward_passes_per_step=1, op=Average)
        random.seed(42)
        mismatches = []
        for s in range(3):
            gen = torch.Generator().manual_seed(900 + 10 * s + rank)
            x = torch.randn(32, 64, generator=gen)
            y = torch.randint(0, 10, (32,), generator=gen)
            loss = torch.nn.functional.cross_entropy(model(x), y)
            loss.backward()
            dopt.step()
            dopt.zero_grad()
            for n, p in model.named_parameters():
                want = golden[f"s{s}/r{rank}/{n}"]
                if not np.array_equal(p.detach().numpy().view(np.uint32), want.view(np.uint32)):
                    mismatches.append((s, n, float(np.abs(p.detach().numpy() - want).max())))
        queue.put((rank, mismatches))
    except Exception as e:  # pragma: no cover - reported to the parent
        queue.put((rank, [("error", repr(e))]))
    finally:
        dist.destroy_process_group()


def _digest(model):
    import hashlib
    h = hashlib.sha256()
    for _, p in model.named_parameters():
        h.update(p.detach().numpy().tobytes())
    return h.hexdigest()


def resnet20_worker(rank, world, port, golden_dir, queue):
    """BASELINE.json configs[0] on the product plumbing: ResNet-20, DGC ratio 0.001 with
    5-epoch warmup, fp16 values, int32 indices, 2 gloo ranks (horovodrun -np 2 in the
    reference). Compared with the reference's per-step parameter digests and final
    weights (tests/golden/optimizer_resnet20.*)."""
    import contextlib
    import io
    import json

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgc.horovod import DistributedOptimizer
        from dgc.optim import DGCSGD
        meta = json.load(open(os.path.join(golden_dir, "optimizer_resnet20.json")))
        final = np.load(os.path.join(golden_dir, "optimizer_resnet20.npz"))
        torch.manual_seed(meta["model_seed"])
        model = ResNet20()
        problems = [] if _digest(model) == meta["init_digest"] else [("init", "digest")]
        opt = DGCSGD(model.parameters(), lr=meta["lr"], momentum=meta["momentum"],
                     weight_decay=meta["weight_decay"], nesterov=meta["nesterov_sgd"])
        mem = OracleMemory(momentum=meta["momentum"])
        with contextlib.redirect_stdout(io.StringIO()):
            comp = OracleDGCCompressor(meta["ratio"], memory=mem, sample_ratio=meta["sample_ratio"],
                                       fp16_values=meta["fp16_values"], int32_indices=meta["int32_indices"],
                                       warmup_epochs=meta["warmup_epochs"])
            mem.initialize(model.named_parameters())
            comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        dopt = DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                    backward_passes_per_step=1, op=Average)
        random.seed(meta["random_seed"])
        spe, batch, s = meta["steps_per_epoch"], meta["batch"], 0
        for ei, e in enumerate((0, 1, 5)):
            with contextlib.redirect_stdout(io.StringIO()):
                comp.warmup_compress_ratio(e)
            if comp.compress_ratio != meta["epoch_ratios"][ei]:
                problems.append(("ratio", e, comp.compress_ratio))
            for _ in range(spe):
                gen = torch.Generator().manual_seed(1900 + 10 * s + rank)
                x = torch.randn(batch, 3, 32, 32, generator=gen)
                y = torch.randint(0, 10, (batch,), generator=gen)
                torch.nn.functional.cross_entropy(model(x), y).backward()
                dopt.step()
                dopt.zero_grad()
                if _digest(model) != meta["step_digests"][s][rank]:
                    problems.append(("step", s))
                s += 1
        for n, p in model.named_parameters():
            want = final[f"final/{n}"]
            if not np.array_equal(p.detach().numpy().view(np.uint32), want.view(np.uint32)):
                problems.append(("final", n, float(np.abs(p.detach().numpy() - want).max())))
        queue.put((rank, problems))
    except Exception as e:  # pragma: no cover - reported to the parent
        queue.put((rank, [("error", repr(e))]))
    finally:
        dist.destroy_process_group()


def comm_worker(rank, world, port, queue):
    """dgc.comm collectives: variable-length allgather, allreduce Average/Sum."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgc import comm
        out = []
        t = torch.arange(rank + 2, dtype=torch.float32).view(-1, 1) + 10 * rank
        g = comm.synchronize(comm.allgather_async(t, name="x"))
        out.append(g.view(-1).tolist())
        a = torch.full((3,), float(rank + 1))
        out.append(comm.synchronize(comm.allreduce_async_(a, name="a", op=comm.Average)).tolist())
        b = torch.full((2,), float(rank + 1))
        out.append(comm.synchronize(comm.allreduce_async_(b, name="b", op=comm.Sum)).tolist())
        out.append((comm.size(), comm.rank()))
        # above RANK_ORDER_MAX: the backend's allreduce (no allgather of W copies)
        calls = {"all_reduce": 0, "all_gather_into_tensor": 0}
        real = {k: getattr(dist, k) for k in calls}

        def counted(k):
            def f(*a, **kw):
                calls[k] += 1
                return real[k](*a, **kw)
            return f
        for k in calls:
            setattr(dist, k, counted(k))
        big = torch.arange(comm.RANK_ORDER_MAX + 5, dtype=torch.float32) * (rank + 1)
        got = comm.synchronize(comm.allreduce_async_(big, name="big", op=comm.Average))
        for k in calls:
            setattr(dist, k, real[k])
        want = torch.arange(comm.RANK_ORDER_MAX + 5, dtype=torch.float32) * sum(range(1, world + 1)) / world
        out.append((got is big, torch.equal(got, want), dict(calls)))
        queue.put((rank, out))
    finally:
        dist.destroy_process_group()


def multi_worker(rank, world, port, golden_dir, label, queue):
    """tests/golden/optimizer_multi.* case ``label`` at its world size: the reference's
    DistributedOptimizer + DGCSGD on TinyNet (W = 3 / 4 / 8, fp32 or fp16 wire values,
    a ratio-1 warmup epoch), run from its data seeds through the product plumbing with the
    oracle doubles; the dense tensors' Average is dgc.comm's rank-order allgather sum."""
    import contextlib
    import io
    import json

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgc.horovod import DistributedOptimizer
        from dgc.optim import DGCSGD
        cfg = json.load(open(os.path.join(golden_dir, "optimizer_multi.json")))[label]
        want = np.load(os.path.join(golden_dir, "optimizer_multi.npz"))
        torch.manual_seed(cfg["model_seed"])
        model = TinyNet()
        opt = DGCSGD(model.parameters(), lr=cfg["lr"], momentum=cfg["momentum"], weight_decay=cfg["weight_decay"],
                     nesterov=cfg["nesterov_sgd"])
        mem = OracleMemory(momentum=cfg["momentum"])
        with contextlib.redirect_stdout(io.StringIO()):
            comp = OracleDGCCompressor(cfg["ratio"], memory=mem, fp16_values=cfg["fp16_values"],
                                       int32_indices=cfg["int32_indices"], **cfg["warmup"])
            mem.initialize(model.named_parameters())
            comp.initialize([(n, p) for n, p in model.named_parameters() if p.dim() > 1])
        dopt = DistributedOptimizer(opt, named_parameters=model.named_parameters(), compression=comp,
                                    backward_passes_per_step=1, op=Average)
        random.seed(cfg["random_seed"])
        spe, problems = cfg["steps_per_epoch"], []
        for ei, e in enumerate(cfg["epochs"]):
            if e is not None:
                with contextlib.redirect_stdout(io.StringIO()):
                    comp.warmup_compress_ratio(e)
            for t in range(spe):
                s = ei * spe + t
                gen = torch.Generator().manual_seed(3000 + 100 * world + 10 * s + rank)
                x = torch.randn(32, 64, generator=gen)
                y = torch.randint(0, 10, (32,), generator=gen)
                torch.nn.functional.cross_entropy(model(x), y).backward()
                dopt.step()
                dopt.zero_grad()
                for n, p in model.named_parameters():
                    w = want[f"{label}/s{s}/{n}"]
                    if not np.array_equal(p.detach().numpy().view(np.uint32), w.view(np.uint32)):
                        problems.append((s, n, float(np.abs(p.detach().numpy() - w).max())))
        queue.put((rank, problems))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        queue.put((rank, [("error", repr(e), traceback.format_exc())]))
    finally:
        dist.destroy_process_group()
