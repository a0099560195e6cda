import sys, os
sys.path[:0] = ["/root/repo", "/root/repo/adam-compression_amd"]
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from oracle import synth
from oracle import torch_cpu as TC
from dgc.memory import DGCSGDMemory
DEV = torch.device("cuda:0")
for dt, scale in ((torch.float16, 1e-2), (torch.float16, 1.0), (torch.bfloat16, 1.0)):
    for nest in (True, False):
        N = 200000
        mem = DGCSGDMemory(momentum=0.9, nesterov=nest)
        mem.initialize([("w", torch.zeros(N, dtype=dt, device=DEV))])
        m = torch.zeros(N, dtype=dt); v = torch.zeros(N, dtype=dt)
        for s in range(2):
            g = torch.from_numpy(synth.gradient(70400 + s, N, "normal", scale).copy()).to(dt)
            mem.compensate(g.to(DEV), "w", accumulate=True)
            TC.compensate(g, m, v, 0.9, nest)
            gm = mem.momentums["w"].cpu(); gv = mem.velocities["w"].cpu()
            bm = (gm.view(torch.int16) != m.view(torch.int16)).nonzero().view(-1)
            bv = (gv.view(torch.int16) != v.view(torch.int16)).nonzero().view(-1)
            print(dt, scale, "nest" if nest else "plain", "step", s, "mmt mism", bm.numel(), "vec mism", bv.numel())
            for i in bm[:3].tolist():
                print("  mmt i", i, "g", g[i].item(), "gpu", gm[i].item(), "cpu", m[i].item())
            for i in bv[:3].tolist():
                print("  vec i", i, "g", g[i].item(), "gpu", gv[i].item(), "cpu", v[i].item(), "mmt", m[i].item())
