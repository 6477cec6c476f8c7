"""Time the two VQ distance paths (vqx_vq_set_path 0 = fp16 MFMA certified +
exact re-rank of uncertified frames, 1 = fp32 MFMA kernel) on data of
different ambiguity: 'clustered' (frames near codebook rows, the trained
regime), 'randn' (independent Gaussians: many near-ties relative to the fp16
bound).  Prints us per call (idx only) and the fraction of frames whose
best / second-best gap is within the certification bound (host fp64 estimate).
Usage: python tools/vq_fast_probe.py [N] [K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import _lib as L, ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
K = int(sys.argv[2]) if len(sys.argv) > 2 else 512
g = torch.Generator().manual_seed(0)


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


for kind in ("clustered", "randn"):
    if kind == "clustered":
        E = torch.randn(K, 128, generator=g) * 1.5
        z = E[torch.randint(0, K, (N,), generator=g)] + 0.3 * torch.randn(N, 128, generator=g)
    else:
        E = torch.randn(K, 128, generator=g)
        z = torch.randn(N, 128, generator=g)
    zd, Ed = z.cuda(), E.cuda()
    d = (zd.double() ** 2).sum(1, keepdim=True) + (Ed.double() ** 2).sum(1)[None] - 2 * zd.double() @ Ed.double().T
    ds = d.topk(2, dim=1, largest=False).values
    nz = zd.double().norm(dim=1)
    ne = Ed.double().norm(dim=1).max()
    delta = 1.0625 * (2 * ((2 ** -10 + 2 ** -16) * nz * ne) + 2 ** -16 * (nz ** 2 + ne ** 2 + 2 * nz * ne))
    amb = ((ds[:, 1] - ds[:, 0]) <= 2 * delta).double().mean().item()
    idx = torch.empty(N, dtype=torch.int64, device="cuda")
    part = torch.empty(ops.vq_workspace(N, K, False), device="cuda")
    res = {}
    for path in (0, 1):
        L.call("vqx_vq_set_path", path)
        res[path] = t_us(lambda: ops.vq_forward(zd, Ed, idx, None, None, None, part, None, None))
    L.call("vqx_vq_set_path", 0)
    print(f"N={N} K={K} {kind:9s} uncertified {100 * amb:5.2f}%  fast {res[0]:7.2f} us  fp32 kernel {res[1]:7.2f} us",
          flush=True)
