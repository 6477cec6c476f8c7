"""How many frames a split-bf16 VQ prefilter could certify.

A prefilter would score z . e as zh.eh + zh.el + zl.eh on bf16 MFMA (z = zh +
zl + rz, |rz| <= 2^-18 |z|, likewise e) and certify a frame's argmin when
its two smallest approximate distances differ by more than twice the
per-frame error bound
    B = 2 (g_split + g_f32) |z| max_k |e_k| + 2^-22 (|z|^2 + max_k |e_k|^2),
    g_split = 3.2 * 2^-18 + (D + 4) * 2^-24   (dropped terms + fp32 accumulation),
    g_f32   = (D + 2) * 2^-24                 (the fp32 kernel's own dot error),
the rest recomputed by the fp32 kernel.  This probe measures, on the bench
step's own z and codebook (vcc20, bf16, 64 x 256, after `--warm` steps), the
exact fp64 top-2 gaps against 2B (a frame certifies for sure when its exact
gap exceeds 4B, and typically when it exceeds 2B), before building the kernel.
Run on the GPU box: python tools/vq_cert_probe.py [--steps 6]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def frac_certified(z, E):
    """(share with exact gap > 4B, > 2B, median gap / B) for fp32 z [N, D], E [K, D]."""
    z64, e64 = z.double(), E.double()
    D = z.shape[1]
    d = (z64.pow(2).sum(1, keepdim=True) + e64.pow(2).sum(1)) - 2 * z64 @ e64.t()
    top2 = torch.topk(d, 2, dim=1, largest=False).values
    gap = top2[:, 1] - top2[:, 0]
    zn = z64.norm(dim=1)
    emax = e64.norm(dim=1).max()
    g_split = 3.2 * 2.0 ** -18 + (D + 4) * 2.0 ** -24
    g_f32 = (D + 2) * 2.0 ** -24
    B = 2 * (g_split + g_f32) * zn * emax + 2.0 ** -22 * (zn.pow(2) + emax ** 2)
    return (float((gap > 4 * B).double().mean()), float((gap > 2 * B).double().mean()),
            float((gap / B).median()), float((gap / (top2[:, 1].abs() + 1e-30)).median()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    from vae_npvc_amd.trainer.basic import Trainer
    cfg = yaml.safe_load(open(os.path.join(ROOT, "vae_npvc_amd", "conf", "vcc20.yaml")))
    cfg["compute_dtype"] = "bf16"
    torch.manual_seed(777)
    np.random.seed(777)
    tr = Trainer(cfg)
    gen = torch.Generator(device="cpu").manual_seed(1234)
    xs = [torch.randn(64, 80, 256, generator=gen).cuda() for _ in range(4)]
    ys = [torch.randint(0, cfg["y_num"], (64, 1), generator=gen).cuda() for _ in range(4)]
    out = []
    for s in range(a.steps):
        tr.train_step((xs[s % 4], ys[s % 4]))
        w = tr.engine._ws[(64, 256, True)]
        E = tr.model.quantizer.embeddings.detach().float()
        c4, c2, med, relgap = frac_certified(w.z.float(), E)
        out.append(dict(step=s + 1, certified_4B=round(c4, 4), certified_2B=round(c2, 4), median_gap_over_B=round(med, 2),
                        median_rel_gap=relgap))
        print(json.dumps(out[-1]), flush=True)
    # the reference VQ fixture's random data for comparison
    from tests.helpers import load_fixture  # noqa: F401  (path check only)
    rng = np.random.Generator(np.random.PCG64(7))
    z = torch.from_numpy(rng.standard_normal((16384, 128)).astype(np.float32))
    E = torch.from_numpy(rng.standard_normal((512, 128)).astype(np.float32))
    c4, c2, med, relgap = frac_certified(z, E)
    print(json.dumps(dict(data="randn z / randn E", certified_4B=round(c4, 4), certified_2B=round(c2, 4),
                          median_gap_over_B=round(med, 2), median_rel_gap=relgap)))


if __name__ == "__main__":
    main()
