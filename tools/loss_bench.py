"""vqx_logloss_fwd_bwd at config 2's shape (B = 64, 80 mel, T = 256; f32 xhat,
bf16 dxhat with 128-column rows), HIP events, us: the 64-frame LDS-tile kernel
(xhat rows of 80 floats) against the flat kernel the call takes for rows of 81
floats (not a multiple of 4).  Usage: python tools/loss_bench.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B, C, T = 64, 80, 256
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(B, C, T, generator=g).cuda()
xh80 = torch.randn(B * T, C, generator=g).cuda()
xh81 = torch.zeros(B * T, 81, device="cuda")
xh81[:, :C] = xh80
dx = torch.empty(B * T, 128, device="cuda", dtype=torch.bfloat16)[:, :C]
loss, part = torch.zeros(1, device="cuda"), torch.empty(1024, device="cuda")


def t_us(fn):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


for p in range(2):
    a = t_us(lambda: ops.logloss_fwd_bwd(x, xh80, 1.0 / (B * T), dx, loss, part))
    b = t_us(lambda: ops.logloss_fwd_bwd(x, xh81[:, :C], 1.0 / (B * T), dx, loss, part))
    print(f"pass {p}: tile {a:6.2f}  flat {b:6.2f} us")
