"""Encoder backward with an injected dL/dz vs float64 autograd of the oracle
encoder, per tensor (max|d|/max|ref| and ||d||/||ref||), for encoders of
0, 1, 2 and 10 residual blocks: localises an encoder-backward error.
Usage (GPU): python tools/enc_bwd_probe.py"""
import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_encoder_bwd import _oracle_grads  # noqa: E402
from tests.helpers import cfg_of, make_trainer  # noqa: E402
from oracle.vqvae_cpu import seeded_batch, seeded_state_dict  # noqa: E402


def run(cfg, tag, B=4, T=128, fuse=None):
    wseed = 11
    sd = seeded_state_dict(cfg, wseed)
    x, y = seeded_batch(cfg, B, T, 5)
    tr = make_trainer(cfg, wseed)
    eng = tr.engine
    torch.manual_seed(0)
    np.random.seed(0)
    w = eng.forward_train(x.cuda().contiguous(), y.cuda())
    Z, Tz = eng.dims["Z"], w.Tz
    g = torch.Generator().manual_seed(99)
    dz = torch.randn(B, Z, Tz, generator=g) / (B * Tz)
    eng.encoder_bwd(w, dz=dz.permute(0, 2, 1).reshape(B * Tz, Z).contiguous().cuda())
    torch.cuda.synchronize()
    ref, z64 = _oracle_grads(cfg, sd, x, dz, torch.float64)
    zh = w.z.view(B, Tz, Z).permute(0, 2, 1).double().cpu()
    print(f"== {tag}: z err {float((zh - z64).abs().max() / z64.abs().max()):.2e}")
    params = dict(tr.model.named_parameters())
    for n, r in ref.items():
        got = eng.g(params[n]).double().cpu().view_as(r)
        mx = float((got - r).abs().max() / r.abs().max().clamp_min(1e-30))
        nr = float((got - r).norm() / r.norm().clamp_min(1e-30))
        print(f"  {n:45s} max {mx:.2e}  norm {nr:.2e}")


if __name__ == "__main__" and not os.environ.get("PROBE_STATS") and not os.environ.get("PROBE_LAST") and not os.environ.get("PROBE_SAVED") and not os.environ.get("PROBE_TRACE"):
    base = cfg_of("vcc20", compute_dtype="fp32")
    for stacks in (0, 1, 2, 10):
        c = copy.deepcopy(base)
        c["encoder"]["stacks"] = [stacks]
        try:
            run(c, f"vcc20 fp32 encoder stacks={stacks}")
        except Exception as e:  # noqa: BLE001
            print(f"== stacks={stacks}: {e!r}")


def check_stats(cfg, B=4, T=128):
    """mean/rstd the forward stored for each block's GroupNorm vs float64 of h."""
    tr = make_trainer(cfg, 11)
    eng = tr.engine
    x, y = seeded_batch(cfg, B, T, 5)
    torch.manual_seed(0)
    np.random.seed(0)
    w = eng.forward_train(x.cuda().contiguous(), y.cuda())
    torch.cuda.synchronize()
    sw = w.enc[0]
    for j in range(len(sw.h)):
        h = sw.h[j][0].double().cpu().view(B, T, -1)
        m = h.mean(dim=(1, 2))
        v = h.var(dim=(1, 2), unbiased=False)
        r = 1.0 / torch.sqrt(v + 1e-5)
        mr = sw.mr[j][0].double().cpu().view(B, 2)
        print(f"  block {j}: |mean| {float(m.abs().max()):.3e} std {float(v.sqrt().max()):.3e}  "
              f"mean err {float((mr[:, 0] - m).abs().max()):.2e}  rstd rel err {float(((mr[:, 1] - r) / r).abs().max()):.2e}")


if __name__ == "__main__" and os.environ.get("PROBE_STATS"):
    c = copy.deepcopy(cfg_of("vcc20", compute_dtype="fp32"))
    check_stats(c)


def check_last_block(cfg, B=4, T=128):
    """The first two launches of encoder_bwd by hand (enc_out DGRAD with the
    GNBWD epilogue for the last block, then that block's GroupNorm backward),
    each checked against float64 torch on the engine's own saved activations."""
    from vae_npvc_amd import ops
    tr = make_trainer(cfg, 11)
    eng = tr.engine
    x, y = seeded_batch(cfg, B, T, 5)
    torch.manual_seed(0)
    np.random.seed(0)
    w = eng.forward_train(x.cuda().contiguous(), y.cuda())
    Z = eng.dims["Z"]
    g = torch.Generator().manual_seed(99)
    dz = (torch.randn(B * T, Z, generator=g) / (B * T)).cuda()
    w.dz.copy_(dz)
    eo = eng.enc_out
    last = w.enc[-1]
    nb = len(last.h)
    k = 0
    cur = eng._enc_cur(w, 0, k)
    w.gnb_part.fill_(float("nan"))
    eng.wgrad_dgrad(eo, w.dz, last.a[-1], cur, last.T, mask=last.a[-1], mask_slope=0.2,
                    **eng._producer_into_enc(w, 0, None, last.cs[-1], True))
    torch.cuda.synchronize()
    W = eo.wp.double().cpu()                       # [128, 512]
    a = last.a[-1].double().cpu()
    ref = (dz.double().cpu() @ W) * torch.where(a > 0, 1.0, 0.2)
    print(f"  cur err {float((cur.double().cpu() - ref).abs().max() / ref.abs().max()):.2e}")
    gn = eng.enc_stages[0].blocks[-1].gns[-1]
    h = last.h[nb - 1][0].double().cpu().view(B, T, -1)
    mr = last.mr[nb - 1][0].double().cpu().view(B, 2)
    xh = (h - mr[:, 0].view(B, 1, 1)) * mr[:, 1].view(B, 1, 1)
    gam = gn.weight.detach().double().cpu()
    dyg = ref.view(B, T, -1) * gam
    s0 = dyg.sum(dim=(1, 2))
    s1 = (dyg * xh).sum(dim=(1, 2))
    C = h.shape[2]
    parts = w.gnb_part[: B * (T // 128) * (C // 128) * 4].double().cpu().view(B, -1, 4).sum(1)
    print(f"  gnbwd s0 err {float((parts[:, 0] - s0).abs().max() / s0.abs().max()):.2e}  "
          f"s1 err {float((parts[:, 1] - s1).abs().max() / s1.abs().max()):.2e}  parts[0]={parts[0].tolist()} "
          f"ref=({float(s0[0]):.4e},{float(s1[0]):.4e})")
    # the block's GroupNorm backward exactly as encoder_bwd runs it
    sw = last
    Cc = sw.C
    dh = type(w).view(w.dh_flat, sw.N, Cc)
    cs_b = eng._bview(w.colsum_b[0], B, Cc)
    dg_b = eng._bview(w.dgam_b[0], B, Cc)
    db_b = eng._bview(w.dbet_b[0], B, Cc)
    nparts = eng._gnb_parts(sw, Cc, True)
    ops.gn_bwd(cur, sw.h[nb - 1][0], dh, sw.T, 1, False, sw.mr[nb - 1][0], gn.weight, gn.bias, w.gnb_part, cs_b, dg_b,
               db_b, nparts=nparts)
    torch.cuda.synchronize()
    n = float(T * C)
    r = mr[:, 1].view(B, 1, 1)
    dh_ref = r * (dyg - (s0 / n).view(B, 1, 1) - xh * (s1 / n).view(B, 1, 1))
    dyv = ref.view(B, T, -1)
    def e(a, b):
        return float((a.double().cpu().reshape(b.shape) - b).abs().max() / b.abs().max())
    print(f"  nparts {nparts}: dh err {e(dh, dh_ref):.2e}  colsum(dh) err {e(cs_b, dh_ref.sum(1)):.2e}  "
          f"dgamma err {e(dg_b, (dyv * xh).sum(1)):.2e}  dbeta err {e(db_b, dyv.sum(1)):.2e}")


if __name__ == "__main__" and os.environ.get("PROBE_LAST"):
    for stacks in (2, 10):
        c = copy.deepcopy(cfg_of("vcc20", compute_dtype="fp32"))
        c["encoder"]["stacks"] = [stacks]
        print(f"== stacks {stacks}")
        check_last_block(c)


def check_saved(cfg, B=4, T=128):
    """Every saved encoder activation after forward_train vs float64 oracle
    intermediates recomputed from x (corruption between forward and backward)."""
    import torch.nn.functional as F
    from oracle.vqvae_cpu import OracleVQVAE
    sd = seeded_state_dict(cfg, 11)
    tr = make_trainer(cfg, 11)
    eng = tr.engine
    x, y = seeded_batch(cfg, B, T, 5)
    torch.manual_seed(0)
    np.random.seed(0)
    w = eng.forward_train(x.cuda().contiguous(), y.cuda())
    torch.cuda.synchronize()
    m = OracleVQVAE(cfg, sd)
    p = {k: v.detach().double() for k, v in m.params.items()}

    def conv(hh, name, pad):
        wv = torch._weight_norm(p[name + ".weight_v"], p[name + ".weight_g"], 0)
        return F.conv1d(hh, wv, p[name + ".bias"], padding=pad)
    sw = w.enc[0]
    c = conv(x.double(), "encoder.encode.0", 1)
    nb = len(sw.h)

    def cmp(tag, got, ref):
        got = got.double().cpu().view(B, T, -1).permute(0, 2, 1)
        print(f"  {tag:10s} err {float((got - ref).abs().max() / ref.abs().max()):.2e}")
    for j in range(nb):
        pre = f"encoder.encode.{j + 1}"
        cmp(f"c[{j}]", sw.c[j], c)
        cmp(f"a[{j}]", sw.a[j], F.leaky_relu(c, 0.2))
        h = conv(F.leaky_relu(c, 0.2), pre + ".stack.1", 1)
        cmp(f"h[{j}]", sw.h[j][0], h)
        c = F.group_norm(h, 1, p[pre + ".stack.2.weight"], p[pre + ".stack.2.bias"], 1e-5) + conv(c, pre + ".skip_layer", 0)
    cmp(f"c[{nb}]", sw.c[nb], c)
    cmp(f"a[{nb}]", sw.a[nb], F.leaky_relu(c, 0.2))


if __name__ == "__main__" and os.environ.get("PROBE_SAVED"):
    for stacks in (2, 10):
        c = copy.deepcopy(cfg_of("vcc20", compute_dtype="fp32"))
        c["encoder"]["stacks"] = [stacks]
        print(f"== stacks {stacks}")
        check_saved(c)


def trace_full(cfg, B=4, T=128):
    """encoder_bwd as the step runs it, with the GroupNorm backward's outputs
    snapshotted right after each gn_bwd and again just before the group's
    weight-norm/column-reduction launch that consumes them."""
    from vae_npvc_amd import ops
    tr = make_trainer(cfg, 11)
    eng = tr.engine
    x, y = seeded_batch(cfg, B, T, 5)
    torch.manual_seed(0)
    np.random.seed(0)
    w = eng.forward_train(x.cuda().contiguous(), y.cuda())
    Z = eng.dims["Z"]
    g = torch.Generator().manual_seed(99)
    dz = (torch.randn(B * T, Z, generator=g) / (B * T)).cuda()
    snaps = []
    real_gn, real_wn = ops.gn_bwd, eng._wn_bwd

    def gn_rec(*a, **k):
        if not snaps:  # the last block's GroupNorm backward: check its inputs like check_last_block
            torch.cuda.synchronize()
            last = w.enc[-1]
            W = eng.enc_out.wp.double().cpu()
            aa = last.a[-1].double().cpu()
            ref = (dz.double().cpu() @ W) * torch.where(aa > 0, 1.0, 0.2)
            cur = a[0].double().cpu()
            print(f"  in-run cur err {float((cur - ref).abs().max() / ref.abs().max()):.2e}  "
                  f"dz err {float((w.dz.double().cpu() - dz.double().cpu()).abs().max()):.2e}  nparts {k.get('nparts')}")
        real_gn(*a, **k)
        torch.cuda.synchronize()
        snaps.append(("gn", [t.detach().clone() for t in a[10:13]]))

    after = {}

    def wn_rec(w_, key):
        torch.cuda.synchronize()
        if after == {} and snaps:
            after["flat"] = None
        if snaps and snaps[-1][0] == "gn":
            now = [t.clone() for t in (eng._bview(w.colsum_b[0], B, 512), eng._bview(w.dgam_b[0], B, 512),
                                       eng._bview(w.dbet_b[0], B, 512))]
            d = [float((a - b).abs().max() / b.abs().max().clamp_min(1e-30)) for a, b in zip(now, snaps[-1][1])]
            print(f"  {key}: cs/dgam/dbet changed between gn_bwd and wn_bwd by {d}")
        real_wn(w_, key)
        torch.cuda.synchronize()
        if key == ("enc", 0, len(w.enc[0].h) - 1):
            after["flat"] = eng.flat_g.detach().clone()
    ops.gn_bwd = gn_rec
    eng._wn_bwd = wn_rec
    try:
        eng.encoder_bwd(w, dz=dz)
    finally:
        ops.gn_bwd = real_gn
    torch.cuda.synchronize()
    sd = seeded_state_dict(cfg, 11)
    dzn = dz.view(B, T, Z).permute(0, 2, 1).cpu()
    # float64 autograd of the encoder with dL/dc_j retained
    import torch.nn.functional as F
    from oracle.vqvae_cpu import OracleVQVAE
    om = OracleVQVAE(cfg, sd)
    pp = {k: v.detach().double().requires_grad_(True) for k, v in om.params.items() if k.startswith("encoder.")}

    def conv(hh, name, pad):
        wv = torch._weight_norm(pp[name + ".weight_v"], pp[name + ".weight_g"], 0)
        return F.conv1d(hh, wv, pp[name + ".bias"], padding=pad)
    nb = len(w.enc[0].h)
    cs = [conv(x.double(), "encoder.encode.0", 1)]
    for j in range(nb):
        pre = f"encoder.encode.{j + 1}"
        cs[-1].retain_grad()
        h = conv(F.leaky_relu(cs[-1], 0.2), pre + ".stack.1", 1)
        cs.append(F.group_norm(h, 1, pp[pre + ".stack.2.weight"], pp[pre + ".stack.2.bias"], 1e-5)
                  + conv(cs[-1], pre + ".skip_layer", 0))
    cs[-1].retain_grad()
    z64 = conv(F.leaky_relu(cs[-1], 0.2), f"encoder.encode.{nb + 2}", 0)
    z64.backward(dzn.double())
    dcl = cs[-1].grad.permute(0, 2, 1).reshape(B * T, -1)
    aa = w.enc[-1].a[-1].double().cpu()
    mine = (dz.double().cpu() @ eng.enc_out.wp.double().cpu()) * torch.where(aa > 0, 1.0, 0.2)
    print(f"  dL/dc_last: autograd vs HIP-activations ref {float((mine - dcl).abs().max() / dcl.abs().max()):.2e}; "
          f"sum err {float((mine.sum(0) - dcl.sum(0)).abs().max() / dcl.sum(0).abs().max()):.2e}; "
          f"bias grad autograd vs this sum {float((pp[f'encoder.encode.{nb}.stack.2.bias'].grad - dcl.sum(0)).abs().max()):.2e}")
    Weo = torch._weight_norm(pp[f"encoder.encode.{nb + 2}.weight_v"], pp[f"encoder.encode.{nb + 2}.weight_g"], 0)
    print(f"  enc_out packed weight vs oracle {float((eng.enc_out.wp.double().cpu() - Weo.detach()[:, :, 0]).abs().max()):.2e}")
    ref, _ = _oracle_grads(cfg, sd, x, dzn, torch.float64)
    params = dict(tr.model.named_parameters())
    nb = len(w.enc[0].h)
    for n, r in ref.items():
        if not n.startswith(f"encoder.encode.{nb}."):
            continue
        p_ = params[n]
        off = (eng.g(p_).data_ptr() - eng.flat_g.data_ptr()) // 4
        mid = after["flat"][off: off + p_.numel()].double().cpu().view_as(r)
        fin = eng.g(p_).double().cpu().view_as(r)
        sc = float(r.abs().max())
        print(f"  {n:40s} right after its group {float((mid - r).abs().max()) / sc:.2e}  at the end {float((fin - r).abs().max()) / sc:.2e}")


if __name__ == "__main__" and os.environ.get("PROBE_TRACE"):
    for stacks in (2, 10):
        c = copy.deepcopy(cfg_of("vcc20", compute_dtype="fp32"))
        c["encoder"]["stacks"] = [stacks]
        print(f"== stacks {stacks}")
        trace_full(c)
