"""How large is the gradient error of a bf16 step INHERENTLY?  Runs the CPU
oracle step twice on the same weights/batch: fp32, and under torch CPU
autocast(bfloat16) (conv/matmul operands rounded to bf16, fp32 accumulation;
the quantizer kept in fp32 like the engine), and prints the per-parameter
relative L2 gradient error of the autocast run against fp32 (median / worst).
Usage: python tools/bf16_autocast_ref.py [vcc20|aishell3] [B] [T]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests.helpers import cfg_of  # noqa: E402
from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "aishell3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
T = int(sys.argv[3]) if len(sys.argv) > 3 else 128
cfg = cfg_of(name)
x, y = seeded_batch(cfg, B, T, 300)
grads = {}
for mode in ("fp32", "bf16"):
    orc = OracleTrainer(dict(cfg), seeded_state_dict(cfg, 91))
    m = orc.model
    if mode == "bf16":
        q0 = m.quantize

        def q_fp32(z, _q=q0):
            with torch.autocast("cpu", enabled=False):
                return _q(z.float())
        m.quantize = q_fp32
    torch.manual_seed(20)
    np.random.seed(20)
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=(mode == "bf16")):
        _, d = orc.train_step((x, y), keep_grads=True)
    grads[mode] = {k: v.double() for k, v in orc.grads.items()}
    print(mode, {k: round(v, 4) for k, v in d.items()})
errs = sorted((float((grads["bf16"][n] - r).norm() / r.norm().clamp_min(1e-30)), n) for n, r in grads["fp32"].items())
print(f"autocast-bf16 vs fp32 step-1 grads: median {errs[len(errs) // 2][0]:.3g} p90 {errs[int(0.9 * len(errs))][0]:.3g}")
for e, n in errs[-6:]:
    print(f"  {e:.3g} {n}")
