"""Shared test helpers (configs, fixtures, seeded trainers)."""
import json
from pathlib import Path

import numpy as np
import torch
import yaml

ROOT = Path(__file__).resolve().parent.parent
GOLD = ROOT / "tests" / "golden"
CONF = ROOT / "vae_npvc_amd" / "conf"


def cfg_of(name, **over):
    cfg = yaml.safe_load(open(CONF / f"{name}.yaml"))
    cfg.update(over)
    return cfg


def load_fixture(prefix):
    meta = json.load(open(GOLD / f"{prefix}.json"))
    arr = dict(np.load(GOLD / f"{prefix}.npz", allow_pickle=False))
    return meta, arr


def relclose(a, b, rtol, atol=0.0):
    return abs(a - b) <= rtol * max(abs(b), 1e-12) + atol


def make_trainer(cfg, wseed):
    from oracle.vqvae_cpu import seeded_state_dict
    from vae_npvc_amd.trainer.basic import Trainer
    torch.manual_seed(0)
    tr = Trainer(cfg)
    tr.model.load_state_dict(seeded_state_dict(cfg, wseed))
    return tr


def oracle_step_grads(cfg, wseed, batch, tseed, nseed, bf16_autocast=False):
    """One oracle train step's (loss dict, per-parameter gradients).  With
    bf16_autocast the conv/matmul operands are rounded to bf16 with fp32
    accumulation (torch CPU autocast) and the quantizer stays fp32 -- the
    engine's bf16 policy restated in stock torch, i.e. the error a bf16 step
    has inherently (tools/bf16_autocast_ref.py)."""
    from oracle.vqvae_cpu import OracleTrainer, seeded_state_dict
    orc = OracleTrainer(dict(cfg, compute_dtype="fp32"), seeded_state_dict(cfg, wseed))
    if bf16_autocast:
        q0 = orc.model.quantize

        def q_fp32(z, _q=q0):
            with torch.autocast("cpu", enabled=False):
                return _q(z.float())
        orc.model.quantize = q_fp32
    torch.manual_seed(tseed)
    np.random.seed(nseed)
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16_autocast):
        _, det = orc.train_step(batch, keep_grads=True)
    return det, {k: v.detach().double() for k, v in orc.grads.items()}


def grad_errors(grads, ref):
    """Sorted per-parameter relative L2 errors [(err, name)] of grads vs ref."""
    out = []
    for n, r in ref.items():
        g = grads[n].detach().double().cpu()
        out.append((float((g - r).norm() / r.norm().clamp_min(1e-30)), n))
    return sorted(out)
