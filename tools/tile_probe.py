"""N < K codebook tiling (layers_vq.py:183-190) of the engine against the
oracle on one step: records each _tile_rows / pick_rows call's input frames
and output rows and the CPU generator state before it, and prints where they
part.  Usage (GPU): python tools/tile_probe.py [B T]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict  # noqa: E402
from tests.helpers import cfg_of, make_trainer  # noqa: E402

B, T = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1, 72)
cfg = cfg_of("vcc20", compute_dtype="fp32")
tr = make_trainer(cfg, 81)
orc = OracleTrainer(cfg, seeded_state_dict(cfg, 81))
x, y = seeded_batch(cfg, B, T, 13)

rec = {"orc": [], "eng": []}
q = orc.model
pick0 = q.pick_rows


def pick(z):
    st = torch.get_rng_state().clone()
    r = pick0(z)
    rec["orc"].append((z.detach().clone(), r.detach().clone(), st))
    return r


q.pick_rows = pick
eng = tr.engine
tile0 = eng._tile_rows


def tile(w):
    st = torch.get_rng_state().clone()
    r = tile0(w)
    rec["eng"].append((w.z.detach().cpu().clone(), r.detach().cpu().clone(), st))
    return r


eng._tile_rows = tile
torch.manual_seed(4)
np.random.seed(4)
orc.train_step((x, y), keep_grads=True)
torch.manual_seed(4)
np.random.seed(4)
tr.train_step((x.cuda(), y.cuda()))
torch.cuda.synchronize()
print("calls", len(rec["orc"]), len(rec["eng"]))
for i, (o, e) in enumerate(zip(rec["orc"], rec["eng"])):
    zo, ro, so = o
    ze, re_, se = e
    print(f"call {i}: z shapes {tuple(zo.shape)} {tuple(ze.shape)} z rel diff "
          f"{float((zo - ze).norm() / zo.norm()):.3g}; rng state equal {bool(torch.equal(so, se))}; "
          f"rows rel diff {float((ro - re_).norm() / ro.norm()):.3g}")
