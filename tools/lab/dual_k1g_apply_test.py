"""The 1x1 data + weight gradient launch with the GroupNorm(/GLU) backward
applied in the same launch (vqx_conv1d_dgrad_wgrad_gnbwd, vqx_gemm_dual.hip
dual_k1g_kernel) against the sequential calls it replaces
(vqx_conv1d_dgrad_wgrad, then vqx_gn_bwd on the GEMM epilogue's partials):
the data gradient, the weight-gradient slabs, the epilogue's partial sums and
the GroupNorm input's gradient bit for bit, the per-utterance column sums to
fp32 rounding (another summation order).  Cases: the decoder res/skip layer
(GLU, GroupNorm G = 2, 640 -> 512 rows), the encoder skip layer (residual +
column sums, G = 1), T = 128 / 256 / 512 (1, 2, 4 row tiles per utterance),
the bench size (64 x 256 frames: the data-gradient grid fills the chip at two
workgroups per CU), repeated calls (the per-utterance counters are left zero),
and the fp32 mode (not fused: the same sequential calls)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _setup(case, B, T, dt, seed=41):
    from vae_npvc_amd import ops
    torch.manual_seed(seed)
    N = B * T
    glu = case == "dec"
    co, ci = (640, 512) if glu else (512, 512)     # forward layer cout, cin
    C = 2 * ci if glu else ci                       # GroupNorm channels
    G = 2 if glu else 1
    dy = torch.randn(N, co, device=DEV).to(dt)
    x = torch.randn(N, ci, device=DEV).to(dt)
    wp = (torch.randn(co, ci, device=DEV) / ci ** 0.5).to(dt)
    u = torch.randn(N, C, device=DEV).to(dt)
    mr = torch.empty(B, G, 2, device=DEV)
    ops.groupnorm_stats(u, T, G, torch.empty(B * G * 24, device=DEV), mr)
    gn = dict(gn_h=u, gn_mr=mr, gn_gamma=torch.randn(C, device=DEV) * 0.5 + 1.0,
              gn_beta=torch.randn(C, device=DEV) * 0.5, gn_groups=G, gn_glu=glu)
    extra = {} if glu else dict(res=torch.randn(N, ci, device=DEV).to(dt))
    splits = 24 if glu else 32
    dkw = dict(T=T, cin=co, cout=ci, ntaps=1, pad=0, **gn, **extra)
    wkw = dict(T=T, r_dim=co, c_dim=ci, ntaps=1, pad=0, shift_sign=1, splits=splits)
    return dict(N=N, B=B, T=T, C=C, ci=ci, co=co, G=G, glu=glu, dy=dy, x=x, wp=wp, dkw=dkw, wkw=wkw,
                splits=splits, colsum=not glu)


def _buffers(s, dt):
    N, B, ci, C = s["N"], s["B"], s["ci"], s["C"]
    nan = float("nan")
    o = {"dx": torch.full((N, ci), nan, device=DEV, dtype=dt),
         "slabs": torch.full((s["splits"], s["co"], ci), nan, device=DEV, dtype=dt),
         "gnb": torch.full((N // 128 * (ci // 128) * 4,), nan, device=DEV),
         "gdx": torch.full((N, C), nan, device=DEV, dtype=dt),
         "cs_b": torch.full((B, C), nan, device=DEV), "dg_b": torch.full((B, C), nan, device=DEV),
         "db_b": torch.full((B, C), nan, device=DEV)}
    if s["colsum"]:
        o["cs"] = torch.full((N // 128, ci), nan, device=DEV)
    return o


def _run(s, dt, fused_call, sync=None):
    from vae_npvc_amd import ops
    o = _buffers(s, dt)
    kw = dict(s["dkw"], gn_bwd=o["gnb"])
    if s["colsum"]:
        kw["colsum"] = o["cs"]
    if fused_call:
        f = ops.conv_dgrad_wgrad_gnbwd(s["dy"], s["wp"], o["dx"], kw, s["dy"], s["x"], o["slabs"], s["wkw"],
                                       o["gdx"], sync, o["cs_b"], o["dg_b"], o["db_b"])
    else:
        ops.conv_dgrad_wgrad(s["dy"], s["wp"], o["dx"], kw, s["dy"], s["x"], o["slabs"], s["wkw"])
        ops.gn_bwd(o["dx"], s["dkw"]["gn_h"], o["gdx"], s["T"], s["G"], s["glu"], s["dkw"]["gn_mr"],
                   s["dkw"]["gn_gamma"], s["dkw"]["gn_beta"], o["gnb"], o["cs_b"], o["dg_b"], o["db_b"],
                   nparts=(s["T"] // 128) * (s["ci"] // 128))
        f = None
    torch.cuda.synchronize()
    return o, f


def _bits(t):
    return t.view(torch.int16) if t.element_size() == 2 else t.view(torch.int32)


def _compare(ref, got, sums_tol):
    for key in ref:
        a, b = ref[key], got[key]
        if key in ("cs_b", "dg_b", "db_b"):
            assert torch.isfinite(b).all(), key
            err = ((a.double() - b.double()).abs().max() / a.double().abs().max().clamp_min(1e-30)).item()
            assert err <= sums_tol, (key, err)
        else:
            if not torch.equal(_bits(a), _bits(b)):
                d = (_bits(a).long() - _bits(b).long()).abs()
                nz = d.nonzero()
                raise AssertionError(f"{key}: {len(nz)} of {d.numel()} differ, max {d.max().item()} ulp, "
                                     f"first at {nz[:8].tolist()}: {a[tuple(nz[0])].item()} vs {b[tuple(nz[0])].item()}")


@pytest.mark.parametrize("case,B,T", [("dec", 4, 256), ("enc", 4, 256), ("dec", 3, 128), ("enc", 2, 512),
                                      ("dec", 2, 512), ("dec", 64, 256), ("enc", 64, 256)])
def test_fused_gn_apply_equals_sequential_calls(case, B, T):
    dt = torch.bfloat16
    s = _setup(case, B, T, dt)
    ref, _ = _run(s, dt, False)
    sync = torch.zeros(2 * B + 4, device=DEV, dtype=torch.int32)
    for rep in range(3):  # the counters must come back to zero after every launch
        got, fused = _run(s, dt, True, sync)
        assert fused, case
        _compare(ref, got, 1e-5)
        assert int(sync.abs().sum().item()) == 0, sync.tolist()


def test_fp32_mode_runs_the_sequential_calls():
    dt = torch.float32
    s = _setup("dec", 2, 256, dt)
    ref, _ = _run(s, dt, False)
    sync = torch.zeros(2 * 2 + 4, device=DEV, dtype=torch.int32)
    got, fused = _run(s, dt, True, sync)
    assert not fused
    _compare(ref, got, 0.0)
