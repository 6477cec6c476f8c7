"""Yardstick: hipBLASLt (torch.matmul, bf16) on the plain GEMMs equivalent to
the config-2 conv layers (im2col already materialised, no epilogue)."""
import torch

SHAPES = {"dec_in (16384x1536 @ 1536x1024)": (16384, 1536, 1024), "enc_k3 (16384x1536 @ 1536x512)": (16384, 1536, 512),
          "enc_sk (16384x512 @ 512x512)": (16384, 512, 512), "dec_rs (16384x512 @ 512x640)": (16384, 512, 640),
          "wgrad dec_in (3072x16384 @ 16384x512)": (3072, 16384, 512), "big (8192^3)": (8192, 8192, 8192)}
for name, (m, k, n) in SHAPES.items():
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 20
    e0.record()
    for _ in range(it):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    print(f"{name:42s} {us:8.1f} us {2 * m * n * k / us / 1e6:8.1f} TFLOP/s", flush=True)
