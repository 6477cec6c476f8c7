"""bf16 engine gradients of one step vs the fp32 oracle's (relative L2 error,
worst parameters and the median), for judging bf16-path numerics changes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.helpers import cfg_of, make_trainer  # noqa: E402
from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict  # noqa: E402

cfg = cfg_of("vcc20", compute_dtype="bf16")
B, T = 4, 128
tr = make_trainer(cfg, 78)
orc = OracleTrainer(dict(cfg), seeded_state_dict(cfg, 78))
x, y = seeded_batch(cfg, B, T, 100)
torch.manual_seed(10)
orc.train_step((x, y), keep_grads=True)
torch.manual_seed(10)
_, d = tr.train_step((x.cuda(), y.cuda()))
dict(d)
errs = []
for n, p in tr.model.named_parameters():
    g = tr.engine.g(p).cpu().double()
    r = orc.grads[n].double()
    errs.append((float((g - r).norm() / r.norm().clamp_min(1e-20)), n))
errs.sort()
print("median", errs[len(errs) // 2][0], "p90", errs[int(len(errs) * 0.9)][0])
for e, n in errs[-6:]:
    print(f"{e:.4e} {n}")
