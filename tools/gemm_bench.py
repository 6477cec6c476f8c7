"""Isolated conv-GEMM timing for profiling: the config-2 layer shapes.
python tools/gemm_bench.py [--iters N] [--only NAME] [--dtype bf16]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import _lib as L  # noqa: E402
from vae_npvc_amd import ops  # noqa: E402

SHAPES = {  # name: (mode, cin, cout, k, prologue)
    "dec_in_fwd": ("fwd", 512, 1024, 3, L.PRO_NONE),
    "enc_k3_fwd": ("fwd", 512, 512, 3, L.PRO_NONE),
    "enc_k3_fwd_pro": ("fwd", 512, 512, 3, L.PRO_LRELU),
    "enc_sk_fwd": ("fwd", 512, 512, 1, L.PRO_NONE),
    "dec_rs_fwd": ("fwd", 512, 640, 1, L.PRO_NONE),
    "dec_in_dgrad": ("dgrad", 512, 1024, 3, L.PRO_NONE),
    "enc_k3_dgrad": ("dgrad", 512, 512, 3, L.PRO_NONE),
    "dec_in_wgrad": ("wgrad", 512, 1024, 3, L.PRO_NONE),
    "enc_k3_wgrad": ("wgrad", 512, 512, 3, L.PRO_NONE),
    "dec_rs_wgrad": ("wgrad", 512, 640, 1, L.PRO_NONE),
    "enc_sk_wgrad": ("wgrad", 512, 512, 1, L.PRO_NONE),
    "fin1_fwd": ("fwd", 80, 80, 1, L.PRO_NONE),
    "enc0_fwd": ("fwd", 80, 512, 3, L.PRO_NONE),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default=None)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--splits", type=int, default=8)
    ap.add_argument("--rotate", type=int, default=1, help="cycle through R operand sets (R*~50 MB > MALL = cold)")
    ap.add_argument("--sweep-splits", default=None, help="comma list: time every wgrad shape at each split count")
    ap.add_argument("--gnstats", action="store_true", help="fwd: GroupNorm statistics tiles in the epilogue (GNSTATS)")
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    B, T = 64, 256
    N = B * T
    dev = "cuda"
    jobs = []
    for name, (mode, cin, cout, k, pro) in SHAPES.items():
        if a.only and a.only not in name:
            continue
        if a.sweep_splits and mode == "wgrad":
            jobs += [(f"{name} s{sp}", mode, cin, cout, k, pro, int(sp)) for sp in a.sweep_splits.split(",")]
        elif not a.sweep_splits:
            jobs.append((name, mode, cin, cout, k, pro, a.splits))
    for name, mode, cin, cout, k, pro, splits in jobs:
        R = a.rotate
        xs = [torch.randn(N, cin, device=dev).to(dt) for _ in range(R)]
        dys = [torch.randn(N, cout, device=dev).to(dt) for _ in range(R)]
        w = (torch.randn(cout, k * cin, device=dev) / (k * cin) ** 0.5).to(dt)
        ys = [torch.empty(N, cout, device=dev, dtype=dt) for _ in range(R)]
        dxs = [torch.empty(N, cin, device=dev, dtype=dt) for _ in range(R)]
        slabs = torch.empty(splits, cout, k * cin, device=dev)
        bias = torch.zeros(cout, device=dev)
        use_gst = a.gnstats and cout % 128 == 0  # GNSTATS tiles need 128-column groups
        gst = torch.empty((N // 128) * ((cout + 127) // 128) * 4, device=dev) if use_gst else None
        fkw = dict(gn_stats=gst, gn_groups=1) if use_gst else {}

        def fn(i):
            x, dy, y, dx = xs[i % R], dys[i % R], ys[i % R], dxs[i % R]
            if mode == "fwd":
                ops.conv_fwd(x, w, y, T=T, cin=cin, cout=cout, ntaps=k, pad=(k - 1) // 2, prologue=pro, bias=bias,
                             **fkw)
            elif mode == "dgrad":
                ops.conv_dgrad(dy, w, dx, T=T, cin=cout, cout=cin, ntaps=k, pad=(k - 1) // 2)
            else:
                ops.conv_wgrad(dy, x, slabs, T=T, r_dim=cout, c_dim=cin, ntaps=k, pad=(k - 1) // 2,
                               q_prologue=pro, splits=splits)
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        flops = 2.0 * N * cin * cout * k
        print(f"{name:14s} {us:8.1f} us  {flops / us / 1e6:8.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
