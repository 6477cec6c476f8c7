"""Weight-norm backward (vqx_weight_norm_bwd) timed per backward group at
config 2 (vcc20, bf16, 64 x 256 frames) after one real train step: the whole
group table, its weight-norm rows alone and its column reductions
(VQX_WN_COLREDUCE: bias / GroupNorm-affine partials) alone.

usage (GPU box): python tools/wn_bwd_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oracle.vqvae_cpu import seeded_batch  # noqa: E402
from tests.helpers import cfg_of, make_trainer  # noqa: E402
from vae_npvc_amd import _lib as L  # noqa: E402
from vae_npvc_amd import ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def sub_table(arr, keep):
    ents = [arr[i] for i in range(len(arr)) if keep(arr[i])]
    if not ents:
        return None
    new = (L.WNLayer * len(ents))(*ents)
    dev = torch.frombuffer(bytearray(bytes(new)), dtype=torch.uint8).to("cuda")
    return new, dev


def main():
    cfg = cfg_of("vcc20", compute_dtype="bf16")
    tr = make_trainer(cfg, 31)
    x, y = seeded_batch(cfg, 64, 256, 41)
    tr.train_step((x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    w = tr.engine._ws[(64, 256, True)]
    tot = 0.0
    for key, tab in w.bwd_tables.items():
        arr, _ = tab
        t_all = timed(lambda: ops.weight_norm_bwd(tab))
        tot += t_all
        rows = sub_table(arr, lambda e: e.kind != L.WN_COLREDUCE)
        cols = sub_table(arr, lambda e: e.kind == L.WN_COLREDUCE)
        t_rows = timed(lambda: ops.weight_norm_bwd(rows)) if rows else 0.0
        t_cols = timed(lambda: ops.weight_norm_bwd(cols)) if cols else 0.0
        desc = " ".join(f"{e.kind}:{e.cout}x{e.cin}x{e.k}/s{e.splits}" for e in arr if e.kind != L.WN_COLREDUCE)
        ncr = sum(1 for e in arr if e.kind == L.WN_COLREDUCE)
        crd = " ".join(f"{e.cin}x{e.cout}" for e in arr if e.kind == L.WN_COLREDUCE)
        print(f"{str(key):22s} all {t_all:6.1f} us | rows {t_rows:6.1f} [{desc}] | {ncr} colreduce {t_cols:6.1f} [{crd}]")
    print(f"sum over groups: {tot:.1f} us")


if __name__ == "__main__":
    main()
