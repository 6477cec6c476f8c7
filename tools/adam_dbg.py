"""Vector (16-B) vs scalar path of vqx_adam_step on the same data, three clipped
steps: mismatch counts and the largest difference per state tensor (the packed
f32 ops differ from the scalar ones by an ulp on some second moments).
usage (GPU box): python tools/adam_dbg.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vae_npvc_amd import ops
DEV = "cuda"
n = 12292
torch.manual_seed(41)
lr, betas, eps, max_norm = 2e-4, (0.5, 0.999), 1e-8, 1.0
p0 = torch.randn(n)
runs = []
for off in (0, 1):
    base = {k: torch.zeros(n + 4, device=DEV) for k in ("p", "g", "m", "v")}
    runs.append(dict({k: t[off:off + n] for k, t in base.items()}, step=torch.zeros(1, dtype=torch.int64, device=DEV),
                     hyper=torch.zeros(16, device=DEV), part=torch.zeros(2048, device=DEV), sumsq=torch.zeros(1, device=DEV)))
    runs[-1]["p"].copy_(p0.to(DEV))
for s in range(3):
    gs = torch.randn(n) * (3.0 if s == 1 else 0.01)
    for r in runs:
        r["g"].copy_(gs.to(DEV))
    ops.grad_sq_norm(runs[0]["g"], runs[0]["part"], runs[0]["sumsq"])
    for r in runs:
        ops.adam_hyper(r["step"], lr, 1.0, 10 ** 9, betas[0], betas[1], eps, r["hyper"])
        ops.adam_step(r["p"], r["g"], r["m"], r["v"], r["hyper"], runs[0]["sumsq"], max_norm)
    torch.cuda.synchronize()
    print("step", s, "sumsq", runs[0]["sumsq"].item(), "hyper equal", torch.equal(runs[0]["hyper"], runs[1]["hyper"]),
          runs[0]["hyper"][:8].tolist())
    for k in ("p", "m", "v"):
        a, b = runs[0][k], runs[1][k]
        d = (a != b).nonzero().flatten()
        print(" ", k, "mismatches", d.numel(), "first", d[:8].tolist(), "maxabs", (a - b).abs().max().item(),
              "nan", torch.isnan(a).sum().item(), torch.isnan(b).sum().item())
