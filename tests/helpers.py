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
