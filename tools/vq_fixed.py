"""Fixed cost of the VQ forward kernel: idx-only time vs K (small K), next to
an 8.4 MB device copy, timed with HIP events (us)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import ops  # noqa: E402

N, D = int(os.environ.get("VQB_N", "16384")), 128
z = torch.randn(N, D, device="cuda")


def t_us(fn, reps=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


y = torch.empty_like(z)
print(f"copy 8.4MB: {t_us(lambda: y.copy_(z)):.2f} us")
idx = torch.empty(N, dtype=torch.int64, device="cuda")
part = torch.empty(ops.vq_workspace(N, 4096, True), device="cuda")
for K in (16, 64, 128, 256, 512, 1024, 2048):
    E = torch.randn(K, D, device="cuda")
    t = t_us(lambda: ops.vq_forward(z, E, idx, None, None, None, part))
    print(f"N={N} K={K:5d} idx-only {t:7.2f} us  ({2.0 * N * K * D / t / 1e6:6.1f} TF)")
