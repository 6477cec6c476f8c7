"""Where the 1x1 layers' time goes (config 2: 16,384 frames): each 1x1 GEMM
of the step timed alone with its real epilogue and with the epilogue
stripped to bias-only, plus the fused DGRAD + WGRAD call, HIP events around
`reps` back-to-back launches on the current stream.
Usage (GPU): python tools/k1_breakdown.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import _lib as L  # noqa: E402
from vae_npvc_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
B, T = 64, 256
N = B * T
dev = "cuda"
bf = torch.bfloat16
g = torch.Generator(device="cpu").manual_seed(0)


def rnd(*s, dt=bf):
    return torch.randn(*s, generator=g).to(dev).to(dt)


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


def row(name, us, flops):
    print(f"{name:44s} {us:7.2f} us  {flops / us / 1e6:7.1f} TF", flush=True)


C, S = 512, 128
# ---- encoder skip 1x1 FWD: c' = GN(h) + W c + b, y2 = LReLU(c')
c, h = rnd(N, C), rnd(N, C)
W = rnd(C, C) / C ** 0.5
bias = torch.zeros(C, device=dev)
y, y2 = torch.empty(N, C, device=dev, dtype=bf), torch.empty(N, C, device=dev, dtype=bf)
mr = torch.empty(B, 2, device=dev)
ops.groupnorm_stats(h, T, 1, torch.empty(B * 64, device=dev), mr)
gam, bet = torch.ones(C, device=dev), torch.zeros(C, device=dev)
fl = 2.0 * N * C * C
row("enc skip FWD bias only", t_us(lambda: ops.conv_fwd(c, W, y, T=T, cin=C, cout=C, ntaps=1, pad=0, bias=bias)), fl)
row("enc skip FWD GNADD + ACT2 (EK3, the step's)",
    t_us(lambda: ops.conv_fwd(c, W, y, T=T, cin=C, cout=C, ntaps=1, pad=0, bias=bias, gn_h=h, gn_mr=mr, gn_gamma=gam,
                              gn_beta=bet, act=L.PRO_LRELU, y2=y2)), fl)
# ---- decoder res/skip 1x1 FWD: [x' | skip] = W g + b, x' += x, skip32 (+)= ...
gg, x = rnd(N, C), rnd(N, C)
Wrs = rnd(C + S, C) / C ** 0.5
brs = torch.zeros(C + S, device=dev)
yrs = torch.empty(N, C, device=dev, dtype=bf)
skip32 = torch.zeros(N, S, device=dev)
yfull = torch.empty(N, C + S, device=dev, dtype=bf)
fl = 2.0 * N * (C + S) * C
row("dec res/skip FWD bias only", t_us(lambda: ops.conv_fwd(gg, Wrs, yfull, T=T, cin=C, cout=C + S, ntaps=1, pad=0,
                                                              bias=brs)), fl)
row("dec res/skip FWD RES + SPLIT (EK2, the step's)",
    t_us(lambda: ops.conv_fwd(gg, Wrs, yrs, T=T, cin=C, cout=C + S, ntaps=1, pad=0, bias=brs, res=x, out2=skip32,
                              split_col=C, out2_accumulate=True)), fl)
# ---- decoder res/skip 1x1 DGRAD (+ GLU/GN backward sums) and WGRAD
dy = rnd(N, C + S)
dg = torch.empty(N, C, device=dev, dtype=bf)
u = rnd(N, 2 * C)
mr2 = torch.empty(B, 4, device=dev)
ops.groupnorm_stats(u, T, 2, torch.empty(B * 2 * 64, device=dev), mr2)
gam2, bet2 = torch.ones(2 * C, device=dev), torch.zeros(2 * C, device=dev)
gnb = torch.empty(N // 128 * 8 * 4, device=dev)
fl = 2.0 * N * (C + S) * C
dk = dict(T=T, cin=C + S, cout=C, ntaps=1, pad=0)
row("dec rs DGRAD plain", t_us(lambda: ops.conv_dgrad(dy, Wrs, dg, **dk)), fl)
glu = dict(gn_bwd=gnb, gn_h=u, gn_mr=mr2, gn_gamma=gam2, gn_beta=bet2, gn_groups=2, gn_glu=True)
row("dec rs DGRAD + GNBWD GLU sums", t_us(lambda: ops.conv_dgrad(dy, Wrs, dg, **dk, **glu)), fl)
splits = 24
slabs = torch.empty(splits, C + S, C, device=dev, dtype=bf)
wk = dict(T=T, r_dim=C + S, c_dim=C, ntaps=1, pad=0, splits=splits)
row("dec rs WGRAD (24 splits, bf16 slabs)", t_us(lambda: ops.conv_wgrad(dy, gg, slabs, **wk)), fl)
row("dec rs DGRAD+GNBWD + WGRAD fused (dual_k1, the step's)",
    t_us(lambda: ops.conv_dgrad_wgrad(dy, Wrs, dg, dict(dk, **glu), dy, gg, slabs, dict(wk, shift_sign=1))), 2 * fl)
du = torch.empty(N, 2 * C, device=dev, dtype=bf)
cs, dgm, dbt = (torch.empty(B, 2 * C, device=dev) for _ in range(3))
row("dec GN/GLU backward apply (vqx_gn_bwd, tiles)",
    t_us(lambda: ops.gn_bwd(dg, u, du, T, 2, True, mr2, gam2, bet2, gnb, cs, dgm, dbt, nparts=(T // 128) * 8)), 0.0 + 1)
# ---- encoder skip 1x1 DGRAD (+ GN(1) backward sums, column sums) and WGRAD
cur = rnd(N, C)
nxt = torch.empty(N, C, device=dev, dtype=bf)
tmp = rnd(N, C)
csp = torch.empty(N // 128, C, device=dev)
gnb1 = torch.empty(N // 128 * 4 * 4, device=dev)
fl = 2.0 * N * C * C
dk1 = dict(T=T, cin=C, cout=C, ntaps=1, pad=0)
row("enc skip DGRAD plain", t_us(lambda: ops.conv_dgrad(cur, W, nxt, **dk1)), fl)
e6 = dict(res=tmp, colsum=csp, gn_bwd=gnb1, gn_h=h, gn_mr=mr, gn_gamma=gam, gn_beta=bet, gn_groups=1)
row("enc skip DGRAD + RES + COLSUM + GNBWD", t_us(lambda: ops.conv_dgrad(cur, W, nxt, **dk1, **e6)), fl)
slabs1 = torch.empty(32, C, C, device=dev, dtype=bf)
wk1 = dict(T=T, r_dim=C, c_dim=C, ntaps=1, pad=0, splits=32)
row("enc skip WGRAD (32 splits)", t_us(lambda: ops.conv_wgrad(cur, c, slabs1, **wk1)), fl)
row("enc skip fused (the step's dual_k1)",
    t_us(lambda: ops.conv_dgrad_wgrad(cur, W, nxt, dict(dk1, **e6), cur, c, slabs1, dict(wk1, shift_sign=1))), 2 * fl)
