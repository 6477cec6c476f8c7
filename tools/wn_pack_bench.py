"""Weight-norm forward (norm + pack into the effective-conv bf16 layout) timed
per layer class at config 2 (vcc20): the engine's own layer table, split by
(kind, v shape), each subset launched alone.  Prints us per launch and the
algorithmic rate (fp32 v read + bf16 w_packed written).

usage (GPU box): python tools/wn_pack_bench.py
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.helpers import cfg_of  # noqa: E402
from vae_npvc_amd import ops  # noqa: E402
from vae_npvc_amd.model.vqvae import Model  # noqa: E402


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    cfg = cfg_of("vcc20", compute_dtype="bf16")
    m = Model(cfg).cuda()
    eng = m.engine(torch.device("cuda"))
    ents = [eng._wn_entry(Lr, bwd=False) for Lr in eng.convs]
    groups = collections.defaultdict(list)
    for e in ents:
        groups[(e["kind"], tuple(e["v"].shape))].append(e)

    def nbytes(es):
        return sum(e["v"].numel() * 4 + e["w_packed"].numel() * e["w_packed"].element_size() for e in es)

    tab = ops.wn_table(ents)
    us = timed(lambda: ops.weight_norm_fwd(tab))
    print(f"all {len(ents)} layers: {us:7.1f} us  {nbytes(ents) / us * 1e-6:6.2f} TB/s")
    for (kind, shp), es in sorted(groups.items(), key=lambda kv: -nbytes(kv[1])):
        t = ops.wn_table(es)
        us = timed(lambda: ops.weight_norm_fwd(t))
        print(f"kind {kind} v{shp} x{len(es):2d}: {us:7.1f} us  {nbytes(es) / us * 1e-6:6.2f} TB/s")


if __name__ == "__main__":
    main()
