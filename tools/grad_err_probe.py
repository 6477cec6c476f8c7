"""Print the fp32 HIP step's per-parameter gradient errors: element-wise vs
the CPU oracle (B=2, T=256) and gradient norms vs the reference golden
step_vcc20 / step_aishell3 -- the data behind the tolerances in
tests/test_gpu_step.py.  Usage (GPU box): python tools/grad_err_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict  # noqa: E402
from tests.helpers import cfg_of, load_fixture, make_trainer  # noqa: E402


def summarize(tag, errs):
    groups = {}
    for n, e in errs.items():
        groups.setdefault(n.split(".")[0], []).append(e)
    for g, v in sorted(groups.items()):
        v = np.array(v)
        print(f"{tag} {g:10s} n={len(v):3d} median {np.median(v):.2e} max {v.max():.2e}", flush=True)
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
    print(f"{tag} worst: " + ", ".join(f"{n}={e:.1e}" for n, e in worst), flush=True)


cfg = cfg_of("vcc20", compute_dtype="fp32")
B, T = 2, 256
tr = make_trainer(cfg, 77)
orc = OracleTrainer(cfg, seeded_state_dict(cfg, 77))
x, y = seeded_batch(cfg, B, T, 5)
torch.manual_seed(9)
orc.train_step((x, y), keep_grads=True)
torch.manual_seed(9)
_, det = tr.train_step((x.cuda(), y.cuda()))
dict(det)
errs = {}
for n, p in tr.model.named_parameters():
    g = tr.engine.g(p).cpu().double()
    r = orc.grads[n].double()
    errs[n] = float((g - r).norm() / r.norm().clamp_min(1e-30))
summarize("oracle-elementwise", errs)

for prefix in ("step_vcc20", "step_aishell3", "step_vcc20_plain", "step_vcc20_plain_nonorm", "step_aishell3_plain",
               "step_vcc20_multi", "step_vcc20_multi_plain"):
    meta, arr = load_fixture(prefix)
    name = prefix[len("step_"):]
    PLAIN = {"vcc20_plain": ("vcc20", {"use_ema": False}),
             "vcc20_plain_nonorm": ("vcc20", {"use_ema": False, "embed_norm": False}),
             "aishell3_plain": ("aishell3", {"use_ema": False})}
    if name in PLAIN:
        c = dict(cfg_of(PLAIN[name][0], compute_dtype="fp32"), **PLAIN[name][1])
    else:
        c = cfg_of(name if "multi" in name else meta["config"], compute_dtype="fp32")
    t2 = make_trainer(c, meta["wseed"])
    torch.manual_seed(meta["tseed"])
    np.random.seed(meta["nseed"])
    xb, yb = seeded_batch(c, meta["B"], meta["T"], meta["bseed"])
    _, d = t2.train_step((xb.cuda(), yb.cuda()))
    dict(d)
    e2 = {}
    for n, p in t2.model.named_parameters():
        gn = float(t2.engine.g(p).double().norm())
        rn = meta["grads"][n]["norm"]
        e2[n] = abs(gn - rn) / max(abs(rn), 1e-30)
    summarize(f"{prefix}-norm", e2)
