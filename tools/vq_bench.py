"""Time vqx_vq_forward variants (full / no EMA statistics / idx only) at
N = 64 x 256 frames, D = 128, K in {128, 512, 1024}, with HIP events on the
launch stream.  Usage: python tools/vq_bench.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
N, D = 16384, 128
g = torch.Generator(device="cpu").manual_seed(0)
z = torch.randn(N, D, generator=g).cuda()


def t_us(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


KS = [int(k) for k in os.environ.get("VQB_K", "128,512,1024").split(",")]
KINDS = os.environ.get("VQB_E", "randn,rows").split(",")
for K in KS:
    for kind in KINDS:
        E = (torch.randn(K, D, generator=g) if kind == "randn" else z[torch.randperm(N, generator=g)[:K]].cpu()).cuda()
        idx = torch.empty(N, dtype=torch.int64, device="cuda")
        zq = torch.empty(N, D, device="cuda")
        zqc = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
        sq = torch.zeros(1, device="cuda")
        part = torch.empty(ops.vq_workspace(N, K, True), device="cuda")
        ema = torch.zeros(K * D + K, device="cuda")
        bs, bc = ema[:K * D].view(K, D), ema[K * D:]
        full = t_us(lambda: ops.vq_forward(z, E, idx, zq, zqc, sq, part, bs, bc))
        nost = t_us(lambda: ops.vq_forward(z, E, idx, zq, zqc, sq, part, None, None))
        only = t_us(lambda: ops.vq_forward(z, E, idx, None, None, None, part, None, None))
        used = int(torch.bincount(idx, minlength=K).gt(0).sum())
        fl = 2.0 * N * K * D
        print(f"K={K:5d} E={kind:5s} used={used:4d}  full {full:7.2f} us ({fl / full / 1e6:6.1f} TF)  "
              f"no-EMA-stats {nost:7.2f}  idx-only {only:7.2f} us  (fp32 MFMA floor {fl / 157.3e12 * 1e6:.2f} us)",
              flush=True)
