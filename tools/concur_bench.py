"""Two independent backward GEMM chains (decoder-like and encoder-like layer
pairs, vqx_conv1d_dgrad_wgrad) on one stream in sequence vs on two streams at
once: does co-running independent launches fill each other's ramps, tails and
epilogue bursts?  usage (GPU box): python tools/concur_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vae_npvc_amd import ops  # noqa: E402

dev = "cuda"
bf = torch.bfloat16
N, T = 16384, 256


def pair(co, ci, k, splits):
    dy = torch.randn(N, co, device=dev).to(bf)
    x = torch.randn(N, ci, device=dev).to(bf)
    wp = (torch.randn(co, k * ci, device=dev) / (k * ci) ** 0.5).to(bf)
    dx = torch.empty(N, ci, device=dev, dtype=bf)
    slabs = torch.empty(splits, co, k * ci, device=dev, dtype=bf)
    dkw = dict(T=T, cin=co, cout=ci, ntaps=k, pad=(k - 1) // 2)
    wkw = dict(T=T, r_dim=co, c_dim=ci, ntaps=k, pad=(k - 1) // 2, shift_sign=1, splits=splits)
    return lambda: ops.conv_dgrad_wgrad(dy, wp, dx, dkw, dy, x, slabs, wkw)


dec = [pair(1024, 512, 3, 8), pair(640, 512, 1, 25)]   # conv_in-like 3-tap pair, res/skip-like 1x1 pair
enc = [pair(512, 512, 3, 16), pair(512, 512, 1, 32)]   # encoder k3 pair, skip pair
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def seq():
    for f in dec * 5 + enc * 5:
        f()


def conc():
    cur = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(cur)
    sa.wait_event(ev)
    sb.wait_event(ev)
    with torch.cuda.stream(sa):
        for f in dec * 5:
            f()
    with torch.cuda.stream(sb):
        for f in enc * 5:
            f()
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    ea.record(sa)
    eb.record(sb)
    cur.wait_event(ea)
    cur.wait_event(eb)


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for r in range(3):
    print(f"rep {r}: sequential {timed(seq):8.1f} us   two streams {timed(conc):8.1f} us  (5 dec + 5 enc layer pairs)")
