"""GroupNorm-GLU forward at config 2's decoder shape (N = 64 x 256 frames,
u: 1024 bf16 channels -> g: 512), HIP events on the launch stream, us:
  tiles   vqx_gn_glu_fwd_tiles (statistics merged from GEMM tiles in every workgroup, the step's path)
  mr      vqx_gn_glu_fwd with precomputed mean / rstd (no merge prologue)
  add     torch.add of the two halves into g: the same 33.5 MB read + 16.8 MB write, a streaming yardstick
  bwd     vqx_gn_bwd, GLU, with 8 GNBWD tiles per utterance (the step's decoder path: 84 MB moved)
  bwd1    vqx_gn_bwd, G = 1 on 512 channels with 8 tiles (the encoder's: 50 MB)
Usage: python tools/gn_bench.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
B, T, C = 64, 256, 1024
N = B * T
gen = torch.Generator(device="cpu").manual_seed(0)
u = torch.randn(N, C, generator=gen).to(torch.bfloat16).cuda()
g = torch.empty(N, C // 2, dtype=torch.bfloat16, device="cuda")
gamma = torch.rand(C, generator=gen).cuda() + 0.5
beta = torch.randn(C, generator=gen).cuda() * 0.1
rg, ntn = T // 128, C // 128
tiles = torch.zeros(B * rg, ntn, 4)
tiles[..., 0] = 128.0 * 128.0
tiles[..., 1] = torch.randn(B * rg, ntn, generator=gen) * 0.1
tiles[..., 2] = 128.0 * 128.0 * (1.0 + torch.rand(B * rg, ntn, generator=gen))
tiles = tiles.cuda()
mr = torch.zeros(B, 4, device="cuda")
ops.gn_glu_fwd_tiles(u, g, T, tiles, mr, gamma, beta)
mr2 = mr.clone()


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


ref = g.clone()
ops.gn_glu_fwd(u, g, T, mr2, gamma, beta)
torch.cuda.synchronize()
same = torch.equal(ref, g)
a, b = u[:, : C // 2], u[:, C // 2:]
dy = torch.randn(N, C // 2, generator=gen).to(torch.bfloat16).cuda()
du = torch.empty_like(u)
parts = torch.randn(B * 8 * 4, generator=gen).cuda()
cs, dgm, dbt = (torch.empty(B, C, device="cuda") for _ in range(3))
h1 = torch.randn(N, C // 2, generator=gen).to(torch.bfloat16).cuda()
dh1 = torch.empty_like(h1)
mr1 = torch.rand(B, 2, generator=gen).cuda() + 0.5
g1, b1 = gamma[: C // 2].contiguous(), beta[: C // 2].contiguous()
for p in range(2):
    print(f"pass {p}: tiles {t_us(lambda: ops.gn_glu_fwd_tiles(u, g, T, tiles, mr, gamma, beta)):6.2f}  "
          f"mr {t_us(lambda: ops.gn_glu_fwd(u, g, T, mr2, gamma, beta)):6.2f}  "
          f"add {t_us(lambda: torch.add(a, b, out=g)):6.2f}  "
          f"bwd {t_us(lambda: ops.gn_bwd(dy, u, du, T, 2, True, mr2, gamma, beta, parts, cs, dgm, dbt, nparts=8)):6.2f}  "
          f"bwd1 {t_us(lambda: ops.gn_bwd(dy, h1, dh1, T, 1, False, mr1, g1, b1, parts, cs, dgm, dbt, nparts=8)):6.2f}"
          f" us   (tiles == mr output: {same})")
