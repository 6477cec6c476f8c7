"""Yardstick: hipBLASLt (torch.matmul) on the plain GEMMs equivalent to the
config-2 conv layers (im2col already materialised, no epilogue, no fusion),
in the operand layouts the step has them (frames-major activations, so a
weight gradient is dy^T @ x).  bf16 for the conv layers, fp32 for the VQ
distance GEMM.  Output: one line per shape, microseconds and TFLOP/s, the
same-box ceiling the hand-written kernels' fractions read against.

usage: python tools/blas_ref.py  (on the GPU box)
"""
import torch

N = 64 * 256  # frames per GPU at config 2
# name: (M, K, Nout, transpose_a) — C[M, Nout] = A[M, K] @ B[K, Nout]
SHAPES = {
    "dec_in FWD   3-tap 512->1024  (N x 1536 @ 1536 x 1024)": (N, 1536, 1024, False),
    "dec_in DGRAD 3-tap 1024->512  (N x 3072 @ 3072 x 512)": (N, 3072, 512, False),
    "dec_in WGRAD 1024 x 1536 over N (dy^T @ xcol)": (1024, N, 1536, True),
    "enc_k3 FWD   3-tap 512->512   (N x 1536 @ 1536 x 512)": (N, 1536, 512, False),
    "enc_k3 DGRAD 3-tap 512->512   (N x 1536 @ 1536 x 512)": (N, 1536, 512, False),
    "enc_k3 WGRAD 512 x 1536 over N": (512, N, 1536, True),
    "enc_sk FWD   1x1 512->512     (N x 512 @ 512 x 512)": (N, 512, 512, False),
    "enc_sk DGRAD 1x1 512->512": (N, 512, 512, False),
    "enc_sk WGRAD 512 x 512 over N": (512, N, 512, True),
    "dec_rs FWD   1x1 512->640     (N x 512 @ 512 x 640)": (N, 512, 640, False),
    "dec_rs DGRAD 1x1 640->512     (N x 640 @ 640 x 512)": (N, 640, 512, False),
    "dec_rs WGRAD 640 x 512 over N": (640, N, 512, True),
    "big 8192^3 (chip ceiling)": (8192, 8192, 8192, False),
}


def time_mm(a, b, it=50):
    for _ in range(5):
        a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        a @ b
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    print(f"# {torch.cuda.get_device_name(0)}, torch {torch.__version__}; bf16 peak 2500 TF, fp32 MFMA 157.3 TF")
    for name, (m, k, n, ta) in SHAPES.items():
        if ta:
            a = torch.randn(k, m, device="cuda", dtype=torch.bfloat16).t()
        else:
            a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
        us = time_mm(a, b)
        tf = 2 * m * n * k / us / 1e6
        print(f"{name:58s} {us:8.1f} us {tf:8.1f} TFLOP/s  frac {tf / 2500:.3f}", flush=True)
    # the VQ distance's dot products: z [N, 128] @ E^T [128, 512], fp32
    z = torch.randn(N, 128, device="cuda")
    e = torch.randn(512, 128, device="cuda")
    us = time_mm(z, e.t())
    tf = 2 * N * 128 * 512 / us / 1e6
    print(f"{'VQ dot fp32 (N x 128 @ 128 x 512), no argmin':58s} {us:8.1f} us {tf:8.1f} TFLOP/s  "
          f"frac {tf / 157.3:.3f} of fp32 MFMA", flush=True)
    # and the torch composition of the reference's distance + argmin (layers_vq.py:285-292)
    def dist_argmin():
        d = (z.pow(2).sum(1, keepdim=True) + e.pow(2).sum(1)) - 2 * (z @ e.t())
        return d.argmin(1)
    for _ in range(5):
        dist_argmin()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        dist_argmin()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 50
    print(f"{'VQ distance + argmin, torch ops (reference formula)':58s} {us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
