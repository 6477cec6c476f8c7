"""Time the batched speaker-conditioning linears (vqx_linear_batched_fwd/bwd)
at config 2's shape (10 layers, B = 64, I = 128, O = 1024) in isolation.
Usage (GPU box): python tools/lin_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import ops  # noqa: E402

n, B, I, O = 10, 64, 128, 1024
g = torch.Generator().manual_seed(0)
c = torch.randn(B, I, generator=g).cuda()
lay = [dict(W=torch.randn(O, I, generator=g).cuda(), bias=torch.randn(O, generator=g).cuda(),
            out=torch.empty(B, O, device="cuda"), dout=torch.randn(B, O, generator=g).cuda(),
            dW=torch.empty(O, I, device="cuda"), dbias=torch.empty(O, device="cuda")) for _ in range(n)]
tab = ops.linear_table(lay)
dc = torch.empty(B, I, device="cuda")
part = torch.empty(n * ((O + 63) // 64) * B * I, device="cuda")


def t_us(fn, reps=200):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


print(f"fwd {t_us(lambda: ops.linear_batched_fwd(tab, c, B, I, O)):.1f} us", flush=True)
print(f"bwd (dW, dbias) {t_us(lambda: ops.linear_batched_bwd(tab, c, B, I, O, None)):.1f} us", flush=True)
print(f"bwd (dW, dbias, dc) {t_us(lambda: ops.linear_batched_bwd(tab, c, B, I, O, dc, part)):.1f} us", flush=True)
