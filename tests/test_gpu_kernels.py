"""Kernel-level parity of libvqx against plain PyTorch fp32/fp64 references of
the same ops (conv fwd / dgrad / wgrad, ConvTranspose packing, VQ argmin).
Runs on the MI355X only (-m gpu)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from vae_npvc_amd import ops
    return ops


@pytest.fixture(params=[0, 1], ids=["auto", "im2col"])
def tile(request):
    """Run a GEMM test under both kernel policies (vqx_conv_args.kernel_policy,
    through ops.kernel_policy): 0 lets 3-tap bf16 layers with T % 128 == 0
    take the tap-reuse kernel, 1 keeps every layer on the implicit-im2col
    kernel."""
    ops = _ops()
    with ops.kernel_policy(request.param):
        yield request.param


def ref_conv(x_ntc, w, B, T, pad, pro=None):
    x = x_ntc.double().view(B, T, -1).permute(0, 2, 1)
    if pro == "lrelu":
        x = F.leaky_relu(x, 0.2)
    elif pro == "relu":
        x = F.relu(x)
    y = F.conv1d(x, w.double(), padding=pad)
    return y.permute(0, 2, 1).reshape(B * T, -1)


def pack(w):  # Conv1d weight [cout, cin, k] -> [cout, k*cin]
    cout, cin, k = w.shape
    return w.permute(0, 2, 1).reshape(cout, k * cin).contiguous()


TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2}


def relerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,pro", [(80, 512, 3, None), (512, 512, 3, "lrelu"), (512, 128, 1, "lrelu"),
                                            (128, 80, 1, "relu"), (512, 640, 1, None), (512, 1024, 3, None)])
def test_conv_fwd(dtype, cin, cout, k, pro, tile):
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(0)
    B, T = 3, 64
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    w = (torch.randn(cout, cin, k, device=DEV) / (cin * k) ** 0.5)
    bias = torch.randn(cout, device=DEV)
    y = torch.empty(B * T, cout, device=DEV, dtype=torch.float32)
    proc = {None: L.PRO_NONE, "lrelu": L.PRO_LRELU, "relu": L.PRO_RELU}[pro]
    ops.conv_fwd(x, pack(w).to(dtype), y, T=T, cin=cin, cout=cout, ntaps=k, pad=(k - 1) // 2, prologue=proc,
                 bias=bias, out_f32=True)
    torch.cuda.synchronize()
    ref = ref_conv(x.float().cpu(), pack(w).to(dtype).float().cpu().view(cout, k, cin).permute(0, 2, 1), B, T,
                   (k - 1) // 2, pro) + bias.double().cpu()
    assert relerr(y, ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k", [(512, 512, 3), (512, 128, 1), (128, 80, 1), (512, 1024, 3), (80, 512, 3)])
def test_conv_dgrad_wgrad(dtype, cin, cout, k, tile):
    ops = _ops()
    torch.manual_seed(1)
    B, T = 2, 128
    pad = (k - 1) // 2
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    dy = torch.randn(B * T, cout, device=DEV).to(dtype)
    w = (torch.randn(cout, cin, k, device=DEV) / (cin * k) ** 0.5).to(dtype).float()
    # reference via autograd in fp64
    xr = x.double().cpu().view(B, T, cin).permute(0, 2, 1).clone().requires_grad_(True)
    wr = w.double().cpu().clone().requires_grad_(True)
    yr = F.conv1d(xr, wr, padding=pad)
    yr.backward(dy.double().cpu().view(B, T, cout).permute(0, 2, 1))
    dx_ref = xr.grad.permute(0, 2, 1).reshape(B * T, cin)
    dw_ref = pack(wr.grad)
    if cin % 8 == 0:
        dx = torch.empty(B * T, cin, device=DEV, dtype=torch.float32)
        ops.conv_dgrad(dy, pack(w).to(dtype), dx, T=T, cin=cout, cout=cin, ntaps=k, pad=pad, out_f32=True)
        torch.cuda.synchronize()
        assert relerr(dx, dx_ref) < TOL[dtype]
    splits = 3
    slabs = torch.empty(splits, cout, k * cin, device=DEV)
    ops.conv_wgrad(dy, x, slabs, T=T, r_dim=cout, c_dim=cin, ntaps=k, pad=pad, splits=splits)
    torch.cuda.synchronize()
    assert relerr(slabs.sum(0), dw_ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,dil,T", [(512, 512, 3, 2, 128), (256, 256, 3, 4, 64), (128, 256, 5, 1, 96),
                                              (80, 128, 5, 1, 64), (64, 128, 3, 8, 40), (128, 128, 7, 1, 64),
                                              (256, 512, 5, 2, 128)])
def test_conv_dilated_and_wide_kernels(dtype, cin, cout, k, dil, T, tile):
    """Dilated convs (dilation 2**j of the residual stacks, vqvae.py:166,274;
    layers.py:143,153,198-200) and 5/7-tap convs (the decoder's default
    kernel_size 5, vqvae.py:228): FWD, DGRAD and WGRAD against fp64 torch
    autograd, padding (k-1)//2*dil as the reference builds them, including
    utterances shorter than the dilated receptive field."""
    ops = _ops()
    torch.manual_seed(cin + k + dil)
    B = 3
    pad = (k - 1) // 2 * dil
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    dy = torch.randn(B * T, cout, device=DEV).to(dtype)
    w = (torch.randn(cout, cin, k, device=DEV) / (cin * k) ** 0.5).to(dtype).float()
    xr = x.double().cpu().view(B, T, cin).permute(0, 2, 1).clone().requires_grad_(True)
    wr = w.double().cpu().clone().requires_grad_(True)
    yr = F.conv1d(xr, wr, padding=pad, dilation=dil)
    yr.backward(dy.double().cpu().view(B, T, cout).permute(0, 2, 1))
    y = torch.empty(B * T, cout, device=DEV)
    ops.conv_fwd(x, pack(w).to(dtype), y, T=T, cin=cin, cout=cout, ntaps=k, pad=pad, dil=dil, out_f32=True)
    dx = torch.empty(B * T, cin, device=DEV)
    ops.conv_dgrad(dy, pack(w).to(dtype), dx, T=T, cin=cout, cout=cin, ntaps=k, pad=(k - 1) * dil - pad, dil=dil,
                   out_f32=True)
    slabs = torch.empty(3, cout, k * cin, device=DEV)
    ops.conv_wgrad(dy, x, slabs, T=T, r_dim=cout, c_dim=cin, ntaps=k, pad=pad, dil=dil, splits=3)
    torch.cuda.synchronize()
    assert relerr(y, yr.detach().permute(0, 2, 1).reshape(B * T, cout)) < TOL[dtype]
    assert relerr(dx, xr.grad.permute(0, 2, 1).reshape(B * T, cin)) < TOL[dtype]
    assert relerr(slabs.sum(0), pack(wr.grad)) < TOL[dtype]
    # the dilated ConvTranspose1d of the ResSkip blocks (conv_in, layers.py:199) as the
    # flipped-tap conv with pad (k-1)*dil - p, and its weight gradient (shift sign -1)
    xt = xr.detach().clone().requires_grad_(True)
    wt = wr.detach().permute(1, 0, 2).contiguous().clone().requires_grad_(True)  # [cin, cout, k]
    yt = F.conv_transpose1d(xt, wt, padding=pad, dilation=dil)
    yt.backward(dy.double().cpu().view(B, T, cout).permute(0, 2, 1))
    wp_t = wt.detach().flip(-1).permute(1, 2, 0).reshape(cout, k * cin).float().to(DEV).to(dtype)
    y2 = torch.empty(B * T, cout, device=DEV)
    ops.conv_fwd(x, wp_t, y2, T=T, cin=cin, cout=cout, ntaps=k, pad=(k - 1) * dil - pad, dil=dil, out_f32=True)
    slabs2 = torch.empty(2, cin, k * cout, device=DEV)
    ops.conv_wgrad(x, dy, slabs2, T=T, r_dim=cin, c_dim=cout, ntaps=k, pad=(k - 1) * dil - pad, dil=dil,
                   shift_sign=-1, splits=2)
    torch.cuda.synchronize()
    assert relerr(y2, yt.detach().permute(0, 2, 1).reshape(B * T, cout)) < TOL[dtype]
    dwt = slabs2.sum(0).view(cin, k, cout).permute(0, 2, 1).flip(-1)
    assert relerr(dwt, wt.grad) < TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_convtranspose_via_weight_norm_pack(dtype, tile):
    """ConvTranspose1d(cin->cout, k3, p1) through the weight-norm pack kernel
    (dim 0 = in-channels) and the conv GEMM, fwd + wgrad(sign -1)."""
    ops = _ops()
    torch.manual_seed(2)
    B, T, cin, cout, k = 2, 64, 128, 512, 3
    v = torch.randn(cin, cout, k, device=DEV)
    g = torch.rand(cin, device=DEV) + 0.5
    wp = torch.empty(cout, k * cin, device=DEV, dtype=dtype)
    norm = torch.empty(cin, device=DEV)
    tab = ops.wn_table([dict(v=v, g=g, w_packed=wp, norm=norm, kind=1, cout=cout, cin=cin, k=k,
                             dtype=ops.dt_code(dtype))])
    ops.weight_norm_fwd(tab)
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    y = torch.empty(B * T, cout, device=DEV)
    ops.conv_fwd(x, wp, y, T=T, cin=cin, cout=cout, ntaps=k, pad=1, out_f32=True)
    torch.cuda.synchronize()
    wt = torch._weight_norm(v.cpu().double(), g.cpu().double().view(cin, 1, 1), 0)
    xr = x.double().cpu().view(B, T, cin).permute(0, 2, 1).clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    yr = F.conv_transpose1d(xr, wr, padding=1)
    assert relerr(y, yr.detach().permute(0, 2, 1).reshape(B * T, cout)) < TOL[dtype]
    du = torch.randn(B * T, cout, device=DEV).to(dtype)
    yr.backward(du.double().cpu().view(B, T, cout).permute(0, 2, 1))
    slabs = torch.empty(2, cin, k * cout, device=DEV)
    ops.conv_wgrad(x, du, slabs, T=T, r_dim=cin, c_dim=cout, ntaps=k, pad=1, shift_sign=-1, splits=2)
    torch.cuda.synchronize()
    # slab[ci][j'*cout + co] = dW[ci][co][k-1-j']
    dwt = slabs.sum(0).view(cin, k, cout).permute(0, 2, 1).flip(-1)
    assert relerr(dwt, wr.grad) < TOL[dtype]


def test_weight_norm_bwd_table_chunks():
    """vqx_weight_norm_bwd over a table longer than one launch's layers
    (kWnMaxL = 256, the host splits it into launches; the engine's batched
    weight-norm backward runs ~150 entries at once): 600 column-reduction
    entries of ragged shapes, each dst the ordered column sum of its src."""
    ops = _ops()
    torch.manual_seed(12)
    srcs, dsts = [], []
    for i in range(600):
        rows, cols = 1 + (i * 7) % 40, 8 + (i * 13) % 120
        srcs.append(torch.randn(rows, cols, device=DEV))
        dsts.append(torch.full((cols,), float("nan"), device=DEV))
    ops.weight_norm_bwd(ops.wn_table([ops.colreduce_entry(s_, d_) for s_, d_ in zip(srcs, dsts)]))
    torch.cuda.synchronize()
    for s_, d_ in zip(srcs, dsts):
        assert relerr(d_, s_.double().sum(0)) < 1e-6


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_weight_norm_pack_layouts(dtype):
    """vqx_weight_norm_fwd over one table of mixed layers (the flat unit grid):
    Conv1d 1x1 (wave-per-row path, incl. an unaligned row length), Conv1d k3/k5
    (row-in-LDS transpose), ConvTranspose1d k3 (vectorised 64 x 32 tile) and
    ragged / k5 ConvT (scalar tile) against torch._weight_norm packed to
    wp[co][j*cin + ci] (ConvT taps flipped).  fp32: 1e-6 relative; bf16: the
    fp32 result rounded to nearest-even exactly, up to 1 ulp where the norm's
    summation order differs."""
    ops = _ops()
    torch.manual_seed(11)
    specs = [(0, 512, 640, 1), (0, 128, 1024, 1), (0, 70, 33, 1), (0, 512, 512, 3), (0, 96, 80, 5),
             (1, 512, 1024, 3), (1, 100, 70, 3), (1, 64, 48, 5), (1, 128, 96, 1)]
    ents, refs = [], []
    for kind, cin, cout, k in specs:
        shape = (cout, cin, k) if kind == 0 else (cin, cout, k)
        v = torch.randn(*shape, device=DEV)
        rows = shape[0]
        g = torch.rand(rows, device=DEV) + 0.5
        wp = torch.empty(cout, k * cin, device=DEV, dtype=dtype)
        norm = torch.empty(rows, device=DEV)
        ents.append(dict(v=v, g=g, w_packed=wp, norm=norm, kind=kind, cout=cout, cin=cin, k=k,
                         dtype=ops.dt_code(dtype)))
        vd, gd = v.double().cpu(), g.double().cpu()
        w = torch._weight_norm(vd, gd.view(rows, 1, 1), 0)
        eff = w.permute(0, 2, 1) if kind == 0 else w.flip(-1).permute(1, 2, 0)  # [co][j][ci]
        refs.append((eff.reshape(cout, k * cin), vd.flatten(1).norm(dim=1)))
    ops.weight_norm_fwd(ops.wn_table(ents))
    torch.cuda.synchronize()
    for (kind, cin, cout, k), e, (ref, nref) in zip(specs, ents, refs):
        got = e["w_packed"].double().cpu()
        assert relerr(e["norm"], nref) < 1e-6, (kind, cin, cout, k)
        if dtype == torch.float32:
            assert relerr(got, ref) < 1e-6, (kind, cin, cout, k)
        else:
            r16 = ref.float().to(torch.bfloat16).double()
            ulp = (r16.abs() * 2.0 ** -7).clamp_min(1e-30)
            assert bool(((got - r16).abs() <= ulp).all()), (kind, cin, cout, k)


@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("K", [128, 512, 1024])
def test_vq_argmin_exact(K, D):
    """vqx_vq_forward at every built code width (vq_forward_kernel<D>):
    indices equal torch's first-minimum argmin of the reference's distance
    order, z_q the gathered codes, sqerr, counts and per-code sums."""
    ops = _ops()
    torch.manual_seed(3)
    N = 4096
    z = torch.randn(N, D)
    E = torch.randn(K, D)
    dist = (z.pow(2).sum(1, keepdim=True) + E.pow(2).sum(1)) - 2 * z @ E.t()
    ref = dist.argmin(1)
    zd, Ed = z.to(DEV), E.to(DEV)
    idx = torch.empty(N, dtype=torch.int64, device=DEV)
    zq = torch.empty(N, D, device=DEV)
    zqc = torch.empty(N, D, device=DEV, dtype=torch.bfloat16)
    sq = torch.zeros(1, device=DEV)
    part = torch.empty(ops.vq_workspace(N, K, True, D), device=DEV)
    bsum = torch.zeros(K, D, device=DEV)
    bcnt = torch.zeros(K, device=DEV)
    ops.vq_forward(zd, Ed, idx, zq, zqc, sq, part, bsum, bcnt)
    torch.cuda.synchronize()
    idx = idx.cpu()
    assert (idx == ref).float().mean().item() == 1.0, (idx != ref).sum()
    assert torch.equal(zq.cpu(), E[ref])
    sq_ref = (E[ref] - z).pow(2).sum()
    assert abs(sq.item() - sq_ref.item()) / sq_ref.item() < 1e-5
    onehot = F.one_hot(ref, K).float()
    assert torch.allclose(bcnt.cpu(), onehot.sum(0))
    assert torch.allclose(bsum.cpu(), onehot.t() @ z, atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("N,K,collapse,D", [(1000, 16, False, 128), (777, 128, True, 128), (16384, 512, True, 128),
                                            (5000, 1024, False, 128), (3001, 2048, False, 128), (33, 512, False, 128),
                                            (777, 128, True, 64), (3001, 2048, False, 64), (1000, 16, False, 256),
                                            (5000, 1024, True, 256)])
def test_vq_ema_statistics_ragged_and_collapsed(N, K, collapse, D):
    """EMA statistics of vqx_vq_forward (update_emb, layers_vq.py:207-211):
    bsum = onehot(idx)^T z and bcnt = code counts, accumulated (+=) into
    nonzero buffers, for ragged N (partial frame groups and chunks), every
    LDS slice width (K 16 .. 2048) and a collapsed codebook where all frames
    pick 2 codes (the round-1 kernel's same-address atomic pile-up case)."""
    ops = _ops()
    torch.manual_seed(N + K)
    z = torch.randn(N, D)
    E = torch.randn(K, D)
    if collapse:
        E[2:] += 50.0  # every frame is nearest to code 0 or 1
    ref = ((z.pow(2).sum(1, keepdim=True) + E.pow(2).sum(1)) - 2 * z @ E.t()).argmin(1)
    idx = torch.empty(N, dtype=torch.int64, device=DEV)
    part = torch.empty(ops.vq_workspace(N, K, True, D), device=DEV)
    bsum0, bcnt0 = torch.randn(K, D), torch.rand(K)
    bsum, bcnt = bsum0.to(DEV), bcnt0.to(DEV)
    sq = torch.zeros(1, device=DEV)
    ops.vq_forward(z.to(DEV), E.to(DEV), idx, None, None, sq, part, bsum, bcnt)
    idx = idx.cpu()
    assert torch.equal(idx, ref)
    onehot = F.one_hot(ref, K).double()
    assert torch.equal(bcnt.cpu(), bcnt0 + onehot.sum(0).float())  # counts are exact; one f32 add
    want = bsum0.double() + onehot.t() @ z.double()
    assert torch.allclose(bsum.cpu().double(), want, atol=1e-3, rtol=1e-5)
    if collapse:
        assert int((onehot.sum(0) > 0).sum()) <= 2


@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("K", [16, 128, 512, 2048])
def test_vq_stats_counts_equal_bincount_skewed(K, D):
    """vq_stats_kernel's per-chunk code counts race-free (the count
    loop read keys[] while the sort's first pass could swap them): bcnt must
    equal torch.bincount exactly and bsum the per-code sums, over many 512-frame
    chunks, for skewed index streams (geometric code popularity, long runs of
    one code, a single code, ragged N), launched repeatedly."""
    ops = _ops()
    g = torch.Generator().manual_seed(K)
    N = 64 * 512 + 37
    z = torch.randn(N, D, generator=g)
    geo = torch.clamp((torch.log(torch.rand(N, generator=g)) / np.log(0.8)).long(), max=K - 1)
    runs = (torch.arange(N) // 97 * 7919) % K
    single = torch.full((N,), K // 3, dtype=torch.int64)
    mixed = torch.where(torch.rand(N, generator=g) < 0.9, torch.zeros(N, dtype=torch.int64),
                        torch.randint(0, K, (N,), generator=g))
    zd = z.to(DEV)
    part = torch.empty(ops.vq_workspace(N, K, True, D), device=DEV)
    for idx in (geo, runs, single, mixed):
        want_c = torch.bincount(idx, minlength=K).float()
        want_s = torch.zeros(K, D, dtype=torch.float64).index_add_(0, idx, z.double())
        idd = idx.to(DEV)
        for _ in range(8):
            bsum = torch.zeros(K, D, device=DEV)
            bcnt = torch.zeros(K, device=DEV)
            ops.vq_stats(zd, idd, K, part, bsum, bcnt)
            assert torch.equal(bcnt.cpu(), want_c)
            assert torch.allclose(bsum.cpu().double(), want_s, atol=2e-3, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("act", ["lrelu", "relu"])
def test_conv_fwd_act_epilogues(dtype, act, tile):
    """ACT (y = act(v)) and ACT2 (y = v, y2 = act(v)): the producer-side
    activation that replaces GEMM prologues (vqvae.py:186-187 LeakyReLU stack
    head, 316-317 final ReLUs)."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(3)
    B, T, cin, cout, k = 2, 96, 512, 512, 3
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    w = (torch.randn(cout, cin, k, device=DEV) / (cin * k) ** 0.5).to(dtype)
    bias = torch.randn(cout, device=DEV)
    code = L.PRO_LRELU if act == "lrelu" else L.PRO_RELU
    y = torch.empty(B * T, cout, device=DEV, dtype=dtype)
    y2 = torch.empty(B * T, cout, device=DEV, dtype=dtype)
    ops.conv_fwd(x, pack(w.float()).to(dtype), y, T=T, cin=cin, cout=cout, ntaps=k, pad=1, bias=bias, act=code, y2=y2)
    y3 = torch.empty(B * T, cout, device=DEV, dtype=dtype)
    ops.conv_fwd(x, pack(w.float()).to(dtype), y3, T=T, cin=cin, cout=cout, ntaps=k, pad=1, bias=bias, act=code)
    torch.cuda.synchronize()
    ref = ref_conv(x.float().cpu(), w.float().cpu(), B, T, 1) + bias.double().cpu()
    aref = F.leaky_relu(ref, 0.2) if act == "lrelu" else F.relu(ref)
    assert relerr(y, ref) < TOL[dtype]
    assert relerr(y2, aref) < TOL[dtype]
    # y2 is act applied to the same rounded pre-activation: exact in the element dtype
    slope = 0.2 if act == "lrelu" else 0.0
    yf = y.float()
    assert torch.equal(y2, torch.where(yf > 0, yf, slope * yf).to(dtype)) or dtype == torch.bfloat16
    assert torch.equal(y3, y2)


@pytest.mark.parametrize("dt_in", [torch.float32, torch.bfloat16, None])
@pytest.mark.parametrize("dt_out", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,cols,lds,ldd", [(16384, 512, 1024, 1024), (300, 128, 128, 136), (7, 13, 13, 20),
                                               (1, 4096, 4096, 4096)])
def test_convert_2d_paths(dt_in, dt_out, rows, cols, lds, ldd):
    """vqx_convert_2d (strided copy with dtype conversion; src None = zero
    fill) on the 8-element chunk path (cols and both leading dimensions
    multiples of 8) and the element path; the destination's padding columns
    are untouched."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(rows + cols)
    src = None if dt_in is None else torch.randn(rows, lds, generator=g).to(DEV, dt_in)[:, :cols]
    dst_full = torch.full((rows, ldd), 3.0, device=DEV, dtype=dt_out)
    dst = dst_full[:, :cols]
    ops.convert_2d(src, dst)
    torch.cuda.synchronize()
    want = torch.zeros(rows, cols, device=DEV, dtype=dt_out) if src is None else src.to(dt_out)
    assert torch.equal(dst, want)
    if ldd > cols:
        assert (dst_full[:, cols:] == 3.0).all()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C,S", [(16384, 512, 256), (16384, 256, 256), (9, 13, 7)])
def test_convert_2d_zero2(dt, rows, C, S):
    """vqx_convert_2d_zero2 (ABI 126): dst = src and zero_dst = 0 in one launch
    (chunk path) or two (widths not multiples of 8), in the layout of the
    decoder's [dL/dx (C) | dL/dskip (S)] buffers."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(rows + C)
    a = torch.randn(rows, C + S, generator=g).to(DEV, dt)
    b = torch.full((rows, C + S), 5.0, device=DEV, dtype=dt)
    want = a[:, C:].clone()
    ops.convert_2d_zero2(a[:, C:], b[:, C:], a[:, :C])
    torch.cuda.synchronize()
    assert torch.equal(b[:, C:], want) and (b[:, :C] == 5.0).all()
    assert not a[:, :C].any() and torch.equal(a[:, C:], want)


@pytest.mark.parametrize("dt_out", [torch.float32, torch.bfloat16])
def test_scale_act_2d(dt_out):
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(4)
    src = torch.randn(300, 128, device=DEV)
    dst = torch.empty(300, 128, device=DEV, dtype=dt_out)
    s = (1.0 / 11) ** 0.5
    ops.scale_act_2d(src, dst, s, L.PRO_RELU)
    torch.cuda.synchronize()
    assert torch.equal(dst, torch.relu(src * s).to(dt_out))


@pytest.mark.parametrize("n_utt,T", [(3, 128), (1, 384), (5, 64)])
def test_dgrad_colsum_partials(n_utt, T, tile):
    """COLSUM epilogue: per-128-frame-group column sums of the stored fp32
    output (the bias gradient of the next layer down), ragged row counts."""
    ops = _ops()
    torch.manual_seed(5)
    cin, cout, k = 512, 256, 3
    N = n_utt * T
    dy = torch.randn(N, cout, device=DEV).to(torch.bfloat16)
    w = (torch.randn(cout, k * cin, device=DEV) / (k * cin) ** 0.5).to(torch.bfloat16)
    res = torch.randn(N, cin, device=DEV).to(torch.bfloat16)  # RES is read in the compute dtype
    dx = torch.empty(N, cin, device=DEV)
    groups = (N + 127) // 128
    part = torch.full((groups, cin), float("nan"), device=DEV)
    ops.conv_dgrad(dy, w, dx, T=T, cin=cout, cout=cin, ntaps=k, pad=1, res=res, out_f32=True, colsum=part)
    torch.cuda.synchronize()
    pad = torch.zeros(groups * 128 - N, cin, device=DEV)
    want = torch.cat([dx, pad]).view(groups, 128, cin).sum(1)
    assert torch.isfinite(part).all()
    assert relerr(part, want) < 1e-5


@pytest.mark.parametrize("sdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("kind,rows,other,k,splits,wn", [(0, 512, 512, 1, 32, True), (0, 640, 512, 1, 25, True),
                                                        (1, 512, 1024, 3, 8, True), (0, 512, 512, 3, 16, True),
                                                        (0, 80, 128, 1, 3, True), (1, 128, 80, 5, 1, True),
                                                        (0, 256, 64, 1, 7, False), (0, 1024, 128, 1, 1, True),
                                                        (0, 77, 1000, 1, 1, True), (0, 77, 200, 1, 2, True)])
def test_weight_norm_bwd_reduces_slabs_like_torch(sdt, kind, rows, other, k, splits, wn):
    """vqx_weight_norm_bwd (wn_bwd_kernel): sums the split-K slabs (fp32 or
    bf16) in a fixed order, maps them to v's layout (Conv1d rows cout: x =
    j*cin + ci; ConvTranspose1d rows cin: x = j'*cout + co, tap k-1-j') and
    forms the weight-norm gradients dv, dg of torch._weight_norm(v, g, 0);
    1x1 rows split their 25-32 slabs over thread groups, wide rows do not;
    short 1x1 rows with little split work (<= 256 columns, e.g. the
    speaker-conditioning linears' 1024 x 128, one slab) take one wave per row,
    longer ones (77 x 1000) the row-block path;
    a plain weight (weight norm removed) gets dW itself."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(21 + rows + k)
    cout, cin = (rows, other) if kind == 0 else (other, rows)
    v = torch.randn(rows, other * k, device=DEV)
    g = torch.rand(rows, device=DEV) + 0.5 if wn else None
    slabs = torch.randn(splits, rows, k * other, device=DEV).to(sdt)
    wp = torch.empty(cout, k * cin, device=DEV, dtype=torch.bfloat16)
    norm = torch.empty(rows, device=DEV)
    dv = torch.full_like(v, float("nan"))
    dg = torch.full((rows,), float("nan"), device=DEV) if wn else None
    ent = dict(v=v, g=g, w_packed=wp, norm=norm, kind=kind, cout=cout, cin=cin, k=k, dtype=L.VQX_BF16,
               splits=splits)
    if wn:
        ops.weight_norm_fwd(ops.wn_table([ent]))
    else:
        norm.fill_(1.0)
    ops.weight_norm_bwd(ops.wn_table([dict(ent, dv=dv, dg=dg, slabs=slabs)]))
    torch.cuda.synchronize()
    S = slabs.double().cpu().sum(0).view(rows, k, other)  # [row][j][c]
    dW = S.permute(0, 2, 1) if kind == 0 else S.flip(1).permute(0, 2, 1)  # v layout [row][c][j]
    dW = dW.reshape(rows, other * k)
    if not wn:
        assert relerr(dv, dW) < 1e-6
        return
    vd = v.double().cpu().requires_grad_(True)
    gd = g.double().cpu().requires_grad_(True)
    torch._weight_norm(vd, gd.view(rows, 1), 0).backward(dW)
    assert relerr(dv, vd.grad) < 1e-5
    assert relerr(dg, gd.grad) < 1e-5


def test_linear_batched_and_colreduce():
    """Batched speaker-conditioning linears (fwd, dW, dbias, dc) and the
    weight-norm backward's column-reduce entries."""
    from vae_npvc_amd import _lib as L
    ops = _ops()
    torch.manual_seed(6)
    n, B, I, O = 4, 16, 128, 1024
    c = torch.randn(B, I, device=DEV)
    Ws = [torch.randn(O, I, device=DEV) / I ** 0.5 for _ in range(n)]
    bs = [torch.randn(O, device=DEV) for _ in range(n)]
    outs = [torch.empty(B, O, device=DEV) for _ in range(n)]
    douts = [torch.randn(B, O, device=DEV) for _ in range(n)]
    dWs = [torch.empty(O, I, device=DEV) for _ in range(n)]
    dbs = [torch.empty(O, device=DEV) for _ in range(n)]
    tab = ops.linear_table([dict(W=Ws[i], bias=bs[i], out=outs[i], dout=douts[i], dW=dWs[i], dbias=dbs[i])
                            for i in range(n)])
    dc = torch.empty(B, I, device=DEV)
    ops.linear_batched_fwd(tab, c, B, I, O)
    ops.linear_batched_bwd(tab, c, B, I, O, dc)
    src = torch.randn(70, 300, device=DEV)
    dst = torch.empty(300, device=DEV)
    ops.weight_norm_bwd(ops.wn_table([ops.colreduce_entry(src, dst)]))
    torch.cuda.synchronize()
    cd = c.double()
    for i in range(n):
        assert relerr(outs[i], cd @ Ws[i].double().t() + bs[i].double()) < 1e-6
        assert relerr(dWs[i], douts[i].double().t() @ cd) < 1e-6
        assert relerr(dbs[i], douts[i].double().sum(0)) < 1e-6
    want_dc = sum(douts[i].double() @ Ws[i].double() for i in range(n))
    assert relerr(dc, want_dc) < 1e-6
    assert relerr(dst, src.double().sum(0)) < 1e-6
    assert L.WN_COLREDUCE == 2


@pytest.mark.parametrize("B", [64, 13, 200])
def test_linear_cond_fast_path_equals_tiled_kernels(B):
    """The fp32-MFMA conditioning kernels (I = 128, B <= 64, 16-B aligned c;
    vqx_misc.hip linear_cond_*) and the 64x64-tiled kernels the same call
    takes for an unaligned c, both against float64 (the config-2 shape: 10
    layers, O = 1024; B = 13 leaves rows of the tiles empty).  Their summation
    orders differ (round 5), so the bar is fp32 rounding: 1e-6 relative."""
    ops = _ops()
    torch.manual_seed(16)
    n, I, O = 10, 128, 1024
    c0 = torch.randn(B, I, device=DEV)
    runs = []
    for off in (0, 1):  # off = 1: c not 16-B aligned -> tiled kernels
        base = torch.zeros(B * I + 4, device=DEV)
        c = base[off:off + B * I].view(B, I)
        c.copy_(c0)
        g = torch.Generator(device="cpu").manual_seed(3)
        lay = [dict(W=(torch.randn(O, I, generator=g) / I ** 0.5).to(DEV), bias=torch.randn(O, generator=g).to(DEV),
                    out=torch.empty(B, O, device=DEV), dout=torch.randn(B, O, generator=g).to(DEV),
                    dW=torch.empty(O, I, device=DEV), dbias=torch.empty(O, device=DEV)) for _ in range(n)]
        tab = ops.linear_table(lay)
        dc = torch.empty(B, I, device=DEV)
        ops.linear_batched_fwd(tab, c, B, I, O)
        ops.linear_batched_bwd(tab, c, B, I, O, dc)
        torch.cuda.synchronize()
        runs.append((lay, dc))
    cd = c0.double()
    for lay, dc in runs:
        for d in lay:
            assert relerr(d["out"], cd @ d["W"].double().t() + d["bias"].double()) < 1e-6
            assert relerr(d["dW"], d["dout"].double().t() @ cd) < 1e-6
            assert relerr(d["dbias"], d["dout"].double().sum(0)) < 1e-6
        assert relerr(dc, sum(d["dout"].double() @ d["W"].double() for d in lay)) < 1e-6
    (la, dca), (lb, dcb) = runs
    assert torch.equal(dca, dcb)  # the data gradient takes the same kernels either way
    # a row's forward output and data gradient do not depend on the batch around it
    # (data-parallel ranks against one process on the global batch)
    if B == 200:
        sub = runs[0][0]
        cs = c0[:64].clone()
        lay64 = [dict(W=d["W"], bias=d["bias"], out=torch.empty(64, O, device=DEV), dout=d["dout"][:64].clone(),
                      dW=torch.empty(O, I, device=DEV), dbias=torch.empty(O, device=DEV)) for d in sub]
        tab = ops.linear_table(lay64)
        dc64 = torch.empty(64, I, device=DEV)
        ops.linear_batched_fwd(tab, cs, 64, I, O)
        ops.linear_batched_bwd(tab, cs, 64, I, O, dc64)
        torch.cuda.synchronize()
        for d, d64 in zip(sub, lay64):
            assert torch.equal(d["out"][:64], d64["out"])
        assert torch.equal(dca[:64], dc64)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("G,cout", [(1, 512), (2, 1024)])
def test_gnstats_epilogue_matches_standalone(dtype, G, cout, tile):
    """GEMM-epilogue GroupNorm statistics (tiles + finalize) = the standalone
    two-pass statistics kernel (nn.GroupNorm, layers.py:154,201)."""
    ops = _ops()
    torch.manual_seed(7)
    B, T, cin = 3, 256, 512
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    w = (torch.randn(cout, 3 * cin, device=DEV) / (3 * cin) ** 0.5).to(dtype)
    bias = torch.randn(cout, device=DEV)
    y = torch.empty(B * T, cout, device=DEV, dtype=dtype)
    tiles = torch.empty(B * T // 128 * (cout // 128) * 4, device=DEV)
    mr_fused = torch.empty(B, G, 2, device=DEV)
    ops.conv_fwd(x, w, y, T=T, cin=cin, cout=cout, ntaps=3, pad=1, bias=bias, gn_stats=tiles, gn_groups=G)
    ops.gn_finalize_tiles(tiles, B * T, T, cout, G, mr_fused)
    mr_ref = torch.empty(B, G, 2, device=DEV)
    ops.groupnorm_stats(y, T, G, torch.empty(B * G * 24, device=DEV), mr_ref)
    yy = y.double().view(B, T, G, cout // G)
    mean = yy.mean(dim=(1, 3))
    rstd = 1.0 / torch.sqrt(yy.var(dim=(1, 3), unbiased=False) + 1e-5)
    torch.cuda.synchronize()
    # fused stats come from the fp32 values before rounding to `dtype`
    tol = 1e-5 if dtype == torch.float32 else 5e-3
    assert relerr(mr_fused[..., 0], mean) < tol and relerr(mr_fused[..., 1], rstd) < tol
    assert relerr(mr_fused, mr_ref) < tol


@pytest.mark.parametrize("glu", [False, True])
def test_gnbwd_epilogue_matches_standalone(glu, tile):
    """GEMM-epilogue GroupNorm-backward sums feeding vqx_gn_bwd(nparts>0) give
    the same du / per-utterance sums as the standalone two-pass backward."""
    ops = _ops()
    torch.manual_seed(8)
    dt = torch.bfloat16
    B, T, cin = 2, 256, 512
    C = 1024 if glu else 512           # GN channels
    cout = C // 2 if glu else C        # dgrad output = dL/d(GN output) (or dL/dg for GLU)
    G = 2 if glu else 1
    dy = torch.randn(B * T, cin, device=DEV).to(dt)
    w = (torch.randn(cin, cout, device=DEV) / cout ** 0.5).to(dt)   # 1x1 conv cout->cin, dgrad gives [N, cout]
    u = torch.randn(B * T, C, device=DEV).to(dt)
    mr = torch.empty(B, G, 2, device=DEV)
    ops.groupnorm_stats(u, T, G, torch.empty(B * G * 24, device=DEV), mr)
    gamma, beta = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    g_out = torch.empty(B * T, cout, device=DEV, dtype=dt)
    parts = torch.empty(B * T // 128 * (cout // 128) * 4, device=DEV)
    ops.conv_dgrad(dy, w, g_out, T=T, cin=cin, cout=cout, ntaps=1, pad=0, gn_bwd=parts, gn_h=u, gn_mr=mr,
                   gn_gamma=gamma, gn_beta=beta, gn_groups=G, gn_glu=glu)
    outs = []
    for nparts, pt in ((0, torch.empty(B * 64 * 2, device=DEV)), ((T // 128) * (cout // 128), parts)):
        du = torch.empty(B * T, C, device=DEV, dtype=dt)
        cs, dgm, dbt = (torch.empty(B, C, device=DEV) for _ in range(3))
        ops.gn_bwd(g_out, u, du, T, G, glu, mr, gamma, beta, pt, cs, dgm, dbt, nparts=nparts)
        outs.append((du, cs, dgm, dbt))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert relerr(a, b) < 2e-2, relerr(a, b)


@pytest.mark.parametrize("case", ["k1_glu", "k1_res", "k1_plain", "tr_mask", "tr_convt", "gen", "tr_full", "k1_full"])
def test_fused_dgrad_wgrad_equals_separate_launches(case):
    """vqx_conv1d_dgrad_wgrad (vqx_gemm_dual.hip: one launch interleaving a
    layer's data- and weight-gradient GEMMs) against vqx_conv1d_wgrad +
    vqx_conv1d_dgrad, bit for bit (the same kernel bodies on the same tiles):
    the decoder res/skip 1x1 (GLU GroupNorm-backward epilogue, 640 rows = an
    uneven split of the two grids), the encoder skip 1x1 (residual + column
    sums + GroupNorm-backward sums), a plain 1x1 (each 1x1 case in the
    default in-sequence, the interleaved and the three-per-CU form), the
    3-tap tap-reuse pair
    with the activation-derivative mask, the ConvTranspose form (shift -1,
    residual + column sums), and an im2col-only layer (cin 80: two launches);
    *_full at the bench size (64 x 256 frames: 512 + 512 workgroups, so the
    256-block interleaved groups are exercised)."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(31)
    dt = torch.bfloat16
    B, T = (64, 256) if case.endswith("_full") else (4, 256)
    N = B * T
    k = 3 if case.startswith("tr") else 1
    cfg = {"k1_glu": (640, 512), "k1_res": (512, 512), "k1_plain": (512, 768), "tr_mask": (1024, 512),
           "tr_convt": (512, 1024), "gen": (80, 512), "tr_full": (1024, 512), "k1_full": (512, 512)}[case]
    co, ci = cfg                                   # forward layer cout, cin
    dy = torch.randn(N, co, device=DEV).to(dt)
    x = torch.randn(N, ci, device=DEV).to(dt)
    wp = (torch.randn(co, k * ci, device=DEV) / (k * ci) ** 0.5).to(dt)
    dkw = dict(T=T, cin=co, cout=ci, ntaps=k, pad=(k - 1) // 2 * (1 if k == 3 else 0))
    sign, r_dim, c_dim, p_op, q_op = 1, co, ci, dy, x
    if case == "tr_convt":
        sign, r_dim, c_dim, p_op, q_op = -1, ci, co, x, dy
    splits = 32 if case == "k1_full" else 8
    slab_shape = (splits, r_dim, k * c_dim)
    wkw = dict(T=T, r_dim=r_dim, c_dim=c_dim, ntaps=k, pad=(k - 1) // 2, shift_sign=sign, splits=splits)
    extra = {}
    if case == "k1_glu":
        u = torch.randn(N, 2 * ci, device=DEV).to(dt)
        mr = torch.empty(B, 2, 2, device=DEV)
        ops.groupnorm_stats(u, T, 2, torch.empty(B * 2 * 24, device=DEV), mr)
        extra = dict(gn_h=u, gn_mr=mr, gn_gamma=torch.randn(2 * ci, device=DEV), gn_beta=torch.randn(2 * ci, device=DEV),
                     gn_groups=2, gn_glu=True)
    elif case == "k1_res":
        u = torch.randn(N, ci, device=DEV).to(dt)
        mr = torch.empty(B, 1, 2, device=DEV)
        ops.groupnorm_stats(u, T, 1, torch.empty(B * 24, device=DEV), mr)
        extra = dict(gn_h=u, gn_mr=mr, gn_gamma=torch.randn(ci, device=DEV), gn_beta=torch.randn(ci, device=DEV),
                     res=torch.randn(N, ci, device=DEV).to(dt))
    elif case in ("tr_mask", "tr_full"):
        extra = dict(mask=torch.randn(N, ci, device=DEV).to(dt), mask_slope=0.2)
    elif case == "tr_convt":
        extra = dict(res=torch.randn(N, ci, device=DEV).to(dt))
    outs = []
    # separate launches, the default fused call (1x1: DGRAD's round first, then WGRAD's)
    for fused_call in ((False, 0), (True, 0)):
        o = {"dx": torch.full((N, ci), float("nan"), device=DEV, dtype=dt),
             "slabs": torch.full(slab_shape, float("nan"), device=DEV, dtype=dt)}
        kw = dict(extra)
        if case in ("k1_glu", "k1_res"):
            o["gnb"] = torch.full((N // 128 * (ci // 128) * 4,), float("nan"), device=DEV)
            kw["gn_bwd"] = o["gnb"]
        if case in ("k1_res", "tr_convt"):
            o["cs"] = torch.full((N // 128, ci), float("nan"), device=DEV)
            kw["colsum"] = o["cs"]
        if fused_call[0]:
            ops.set_kernel_policy(fused_call[1])
            try:
                fused = ops.conv_dgrad_wgrad(dy, wp, o["dx"], dict(dkw, **kw), p_op, q_op, o["slabs"], wkw)
            finally:
                ops.set_kernel_policy(0)
            assert fused == (case != "gen"), (case, fused)
        else:
            ops.conv_wgrad(p_op, q_op, o["slabs"], **wkw)
            ops.conv_dgrad(dy, wp, o["dx"], **dkw, **kw)
        torch.cuda.synchronize()
        outs.append(o)
    for other in outs[1:]:
        for key in outs[0]:
            a, b = outs[0][key], other[key]
            assert torch.equal(a.view(torch.int16) if a.dtype == dt else a.view(torch.int32),
                               b.view(torch.int16) if b.dtype == dt else b.view(torch.int32)), (case, key)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("glu,C,T", [(True, 1024, 256), (True, 256, 200), (False, 512, 256), (False, 128, 72)])
def test_gn_bwd_matches_torch_autograd(dtype, glu, C, T):
    """vqx_gn_bwd (GroupNorm [+ tanh*sigmoid GLU] backward: du and the
    per-utterance sums of du, dh*xhat and dh) against fp64 torch autograd of
    GroupNorm(G) -> GLU on the same operands and statistics, per utterance.
    T = 200 / 72 exercise the odd trailing row of the two-rows-in-flight loop."""
    ops = _ops()
    torch.manual_seed(21)
    B = 3
    G = 2 if glu else 1
    u = torch.randn(B * T, C, device=DEV).to(dtype)
    cout = C // 2 if glu else C
    dy = torch.randn(B * T, cout, device=DEV).to(dtype)
    gamma, beta = torch.randn(C, device=DEV) * 0.5 + 1.0, torch.randn(C, device=DEV) * 0.5
    mr = torch.empty(B, G, 2, device=DEV)
    ops.groupnorm_stats(u, T, G, torch.empty(B * G * 64, device=DEV), mr)
    du = torch.empty(B * T, C, device=DEV, dtype=dtype)
    cs, dgm, dbt = (torch.empty(B, C, device=DEV) for _ in range(3))
    ops.gn_bwd(dy, u, du, T, G, glu, mr, gamma, beta, torch.empty(B * 32 * 4, device=DEV), cs, dgm, dbt)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    for b in range(B):
        ub = u[b * T:(b + 1) * T].double().cpu().requires_grad_(True)
        gm = gamma.double().cpu().requires_grad_(True)
        bt = beta.double().cpu().requires_grad_(True)
        h = F.group_norm(ub.t().unsqueeze(0), G, gm, bt, eps=1e-5)[0].t()
        h.retain_grad()
        out = torch.tanh(h[:, :C // 2]) * torch.sigmoid(h[:, C // 2:]) if glu else h
        out.backward(dy[b * T:(b + 1) * T].double().cpu())
        assert relerr(du[b * T:(b + 1) * T], ub.grad) < tol, (b, relerr(du[b * T:(b + 1) * T], ub.grad))
        assert relerr(cs[b], ub.grad.sum(0)) < tol
        assert relerr(dgm[b], gm.grad) < tol
        assert relerr(dbt[b], bt.grad) < tol


@pytest.mark.parametrize("mode", ["fwd", "dgrad"])
@pytest.mark.parametrize("n_utt,T,cin,cout", [(1, 128, 512, 512), (3, 128, 512, 1024), (2, 256, 1024, 512),
                                               (1, 384, 128, 512), (2, 256, 512, 80), (2, 256, 80, 512),
                                               (1, 256, 512, 208), (1, 128, 48, 256)])
def test_conv_tap_reuse_matches_im2col_and_fp64(mode, n_utt, T, cin, cout):
    """The tap-reuse kernel (vqx_gemm_kernel.h conv_tr_kernel: one staged
    130-frame window for all three taps, halo frames zeroed at utterance
    edges) against the implicit-im2col kernel on the same bf16 operands and
    against fp64 torch, with a bias + residual epilogue and fp32 output.  K
    sides of 80, 208 and 48 channels (cin % 32 != 0: 16-channel stages, e.g.
    the 80-mel input conv) run the same kernel with BKC = 16."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(7)
    N = n_utt * T
    k_in, k_out = (cin, cout) if mode == "fwd" else (cout, cin)  # GEMM K side / output channels
    a = torch.randn(N, k_in, device=DEV).to(torch.bfloat16)
    w = (torch.randn(cout, cin, 3, device=DEV) / (cin * 3) ** 0.5).to(torch.bfloat16).float()
    wp = pack(w).to(torch.bfloat16)
    bias = torch.randn(k_out, device=DEV)
    res = torch.randn(N, k_out, device=DEV).to(torch.bfloat16)
    outs = []
    for policy in (0, 1):
        ops.set_kernel_policy(policy)
        y = torch.empty(N, k_out, device=DEV, dtype=torch.float32)
        if mode == "fwd":
            ops.conv_fwd(a, wp, y, T=T, cin=cin, cout=cout, ntaps=3, pad=1, bias=bias, res=res, out_f32=True)
        else:
            ops.conv_dgrad(a, wp, y, T=T, cin=cout, cout=cin, ntaps=3, pad=1, bias=bias, res=res, out_f32=True)
        torch.cuda.synchronize()
        outs.append(y)
    ops.set_kernel_policy(0)
    ad = a.double().cpu().view(n_utt, T, k_in).permute(0, 2, 1)
    if mode == "fwd":
        ref = F.conv1d(ad, w.double().cpu(), padding=1)
    else:
        ref = F.conv_transpose1d(ad, w.double().cpu(), padding=1)
    ref = ref.permute(0, 2, 1).reshape(N, k_out) + bias.double().cpu() + res.double().cpu()
    assert relerr(outs[0], outs[1]) < 1e-5  # same bf16 products, fp32 sums in another order
    assert relerr(outs[0], ref) < 2e-5


@pytest.mark.parametrize("mode", ["fwd", "dgrad"])
@pytest.mark.parametrize("n_utt,T,cin,cout", [(2, 256, 512, 512), (1, 512, 512, 1024), (4, 256, 1024, 512),
                                               (2, 768, 128, 224), (8, 256, 512, 1024)])
def test_conv_tall_tap_reuse_matches_tap_reuse_and_fp64(mode, n_utt, T, cin, cout):
    """The tall tap-reuse kernels (256 frames: vqx_gemm_kernel.h
    conv_tr8_kernel; 512 frames: vqx_gemm_pp.h conv_pp_kernel, whose two
    4-wave groups alternate loading and multiplying; 128 columns per 8-wave
    workgroup, one staged window with halo rows per 256-frame segment) against
    the 128-frame tap-reuse kernel and fp64
    torch: segments that start / end utterances and segments whose halo frames
    belong to the same utterance (T = 512, 768), ragged columns (224), and the
    fused epilogues the engine runs on it (bias + residual, GroupNorm
    statistics tiles in FWD, column sums in DGRAD)."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(17)
    N = n_utt * T
    k_in, k_out = (cin, cout) if mode == "fwd" else (cout, cin)
    a = torch.randn(N, k_in, device=DEV).to(torch.bfloat16)
    w = (torch.randn(cout, cin, 3, device=DEV) / (cin * 3) ** 0.5).to(torch.bfloat16).float()
    wp = pack(w).to(torch.bfloat16)
    bias = torch.randn(k_out, device=DEV)
    res = torch.randn(N, k_out, device=DEV).to(torch.bfloat16)
    tn = -(-k_out // 128)
    outs = []
    policies = [4, 2] + ([3] if N % 512 == 0 else [])
    for policy in policies:
        ops.set_kernel_policy(policy)
        y = torch.empty(N, k_out, device=DEV, dtype=torch.float32)
        y2 = torch.empty(N, k_out, device=DEV, dtype=torch.bfloat16)
        red = torch.full((N // 128, tn * 4 if mode == "fwd" else k_out), float("nan"), device=DEV)
        call = ops.conv_fwd if mode == "fwd" else ops.conv_dgrad
        kw = dict(T=T, cin=k_in, cout=k_out, ntaps=3, pad=1)
        call(a, wp, y, bias=bias, res=res, out_f32=True, **kw)
        if mode == "fwd" and k_out % 128 == 0:
            call(a, wp, y2, bias=bias, gn_stats=red, gn_groups=k_out // 128 if k_out <= 512 else 2, **kw)
        elif mode == "dgrad":
            call(a, wp, y2, bias=bias, colsum=red, **kw)
        torch.cuda.synchronize()
        outs.append((y, y2, red))
    ops.set_kernel_policy(0)
    ad = a.double().cpu().view(n_utt, T, k_in).permute(0, 2, 1)
    ref = F.conv1d(ad, w.double().cpu(), padding=1) if mode == "fwd" else \
        F.conv_transpose1d(ad, w.double().cpu(), padding=1)
    ref = ref.permute(0, 2, 1).reshape(N, k_out) + bias.double().cpu()
    for y, y2, red in outs:
        assert relerr(y, ref + res.double().cpu()) < 2e-5
        assert relerr(y, outs[0][0]) < 1e-5
        if mode == "dgrad" or k_out % 128 == 0:
            assert relerr(y2.float(), outs[0][1].float()) < 1e-2  # one bf16 rounding apart at most
            assert relerr(red, outs[0][2]) < 1e-4, (red - outs[0][2]).abs().max()
    if mode == "dgrad":  # per-128-frame column sums of the stored bf16 output
        cs = outs[-1][1].double().cpu().view(N // 128, 128, k_out).sum(1)
        assert relerr(outs[-1][2], cs) < 5e-3  # fp32 sums of the values before their bf16 rounding


@pytest.mark.parametrize("k,T,r_dim,c_dim,splits", [(3, 256, 512, 1024, 8), (1, 256, 640, 512, 25), (3, 96, 128, 80, 3),
                                                     (5, 128, 256, 512, 4)])
def test_wgrad_bf16_slabs_match_fp32_slabs(k, T, r_dim, c_dim, splits):
    """bf16 split-K slabs (vqx_wgrad_args.slab_dtype, the bf16 step's default):
    each split's fp32 partial rounded once to bf16.  Their fp32 sum stays
    within 2e-3 of the fp32 slabs' sum on the tap-reuse, 1x1, generic
    (T % 64 != 0) and 5-tap paths, and the bf16 slab bytes are exactly the
    fp32 partials rounded to nearest-even."""
    ops = _ops()
    torch.manual_seed(13)
    N = 4 * T
    p = torch.randn(N, r_dim, device=DEV).to(torch.bfloat16)
    q = torch.randn(N, c_dim, device=DEV).to(torch.bfloat16)
    kw = dict(T=T, r_dim=r_dim, c_dim=c_dim, ntaps=k, pad=(k - 1) // 2, splits=splits)
    s32 = torch.full((splits, r_dim, k * c_dim), float("nan"), device=DEV)
    s16 = torch.full((splits, r_dim, k * c_dim), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.conv_wgrad(p, q, s32, **kw)
    ops.conv_wgrad(p, q, s16, **kw)
    torch.cuda.synchronize()
    assert torch.equal(s16, s32.to(torch.bfloat16))
    assert relerr(s16.float().sum(0), s32.sum(0)) < 2e-3


@pytest.mark.parametrize("sign", [1, -1])
@pytest.mark.parametrize("n_utt,T,r_dim,c_dim,splits", [(2, 128, 512, 512, 3), (3, 64, 80, 192, 2), (1, 256, 128, 64, 4),
                                                         (2, 256, 1024, 512, 5), (4, 64, 256, 128, 16),
                                                         (3, 192, 256, 128, 1), (1, 256, 72, 256, 3)])
def test_wgrad_tap_reuse_matches_im2col_and_fp64(sign, n_utt, T, r_dim, c_dim, splits):
    """The tap-reuse weight gradients (vqx_gemm_kernel.h wgrad_tr_kernel:
    128 r x 3 taps x 64 c tiles, one staged 66-frame q window per K-tile)
    against the implicit-im2col kernel and fp64, for both shift signs (Conv1d
    and ConvTranspose1d), partial r tiles, empty splits and K-tiles that
    start or end utterances."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(11)
    N = n_utt * T
    p = torch.randn(N, r_dim, device=DEV).to(torch.bfloat16)
    q = torch.randn(N, c_dim, device=DEV).to(torch.bfloat16)
    units = ops.wgrad_tiles(N, T, r_dim, c_dim, 3, 1, L.VQX_BF16)
    assert units == -(-r_dim // 128) * (c_dim // 64)
    outs = []
    # policy 0: the library's pick (tap reuse), 1: implicit im2col
    for policy in (0, 1):
        ops.set_kernel_policy(policy)
        slabs = torch.full((splits, r_dim, 3 * c_dim), float("nan"), device=DEV)
        ops.conv_wgrad(p, q, slabs, T=T, r_dim=r_dim, c_dim=c_dim, ntaps=3, pad=1, shift_sign=sign, splits=splits)
        torch.cuda.synchronize()
        outs.append(slabs.sum(0))
    ops.set_kernel_policy(0)
    pd = p.double().cpu().view(n_utt, T, r_dim)
    qd = q.double().cpu().view(n_utt, T, c_dim)
    ref = torch.zeros(r_dim, 3, c_dim, dtype=torch.float64)
    for j in range(3):
        sh = sign * (j - 1)
        lo, hi = max(0, -sh), min(T, T - sh)
        ref[:, j] = torch.einsum("btr,btc->rc", pd[:, lo:hi], qd[:, lo + sh:hi + sh])
    ref = ref.reshape(r_dim, 3 * c_dim)
    assert relerr(outs[0], outs[1]) < 1e-5
    assert relerr(outs[0], ref) < 2e-5


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("B,T", [(2, 128), (64, 256)])
def test_split_epilogue_with_narrow_residual(acc, B, T, tile):
    """res/skip output split (decoder res_skip layer, layers.py:244-249): the
    GEMM's columns >= split_col go to the fp32 skip accumulator and only the
    first split_col columns take the residual, whose buffer is exactly
    split_col wide (no read past it on the split columns).  At config 2
    (64 x 256 frames: 640 tiles, more than one round of two workgroups per CU)
    the automatic policy runs conv_gemm3_kernel (three per CU); its outputs
    equal the implicit-im2col kernel's bit for bit."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(5)
    cin, C, S = 512, 512, 128
    N = B * T
    x = torch.randn(N, cin, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C + S, cin, 1, device=DEV) / cin ** 0.5).to(torch.bfloat16)
    bias = torch.randn(C + S, device=DEV)
    res = torch.randn(N, C, device=DEV).to(torch.bfloat16)  # exactly split_col wide
    skip0 = torch.randn(N, S, device=DEV)
    outs = []
    for policy in ((0, 1) if tile == 0 else (tile,)):
        ops.set_kernel_policy(policy)
        skip = skip0.clone()
        y = torch.empty(N, C, device=DEV, dtype=torch.bfloat16)
        ops.conv_fwd(x, pack(w.float()).to(torch.bfloat16), y, T=T, cin=cin, cout=C + S, ntaps=1, pad=0, bias=bias,
                     res=res, out2=skip, split_col=C, out2_accumulate=acc)
        torch.cuda.synchronize()
        outs.append((y, skip))
    ops.set_kernel_policy(tile)
    y, skip = outs[0]
    full = x.double().cpu() @ w.double().cpu()[:, :, 0].t() + bias.double().cpu()
    assert relerr(y, full[:, :C] + res.double().cpu()) < 2e-2
    assert relerr(skip, full[:, C:] + (skip0.double().cpu() if acc else 0)) < 2e-2
    for y2, skip2 in outs[1:]:
        assert torch.equal(y, y2) and torch.equal(skip, skip2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T", [(3, 256), (2, 128), (1, 384), (1, 2048)])
def test_gn_glu_fwd_tiles_equals_finalize_then_glu(dtype, B, T):
    """vqx_gn_glu_fwd_tiles (statistics merged from the GEMM's GNSTATS tiles
    inside the GLU launch) = vqx_gn_finalize_tiles + vqx_gn_glu_fwd, bit for
    bit, including the mean/rstd it writes for the backward.  T = 2048 has 64
    tiles per group: the merge reads them from memory instead of shuffling."""
    ops = _ops()
    torch.manual_seed(9)
    cin, cout = 512, 1024
    x = torch.randn(B * T, cin, device=DEV).to(dtype)
    w = (torch.randn(cout, 3 * cin, device=DEV) / (3 * cin) ** 0.5).to(dtype)
    bias = torch.randn(cout, device=DEV)
    gamma, beta = torch.randn(cout, device=DEV), torch.randn(cout, device=DEV)
    u = torch.empty(B * T, cout, device=DEV, dtype=dtype)
    tiles = torch.empty(B * T // 128 * (cout // 128) * 4, device=DEV)
    ops.conv_fwd(x, w, u, T=T, cin=cin, cout=cout, ntaps=3, pad=1, bias=bias, gn_stats=tiles, gn_groups=2)
    mr1, mr2 = torch.empty(B, 2, 2, device=DEV), torch.full((B, 2, 2), float("nan"), device=DEV)
    g1 = torch.empty(B * T, cout // 2, device=DEV, dtype=dtype)
    g2 = torch.empty_like(g1)
    ops.gn_finalize_tiles(tiles, B * T, T, cout, 2, mr1)
    ops.gn_glu_fwd(u, g1, T, mr1, gamma, beta)
    ops.gn_glu_fwd_tiles(u, g2, T, tiles, mr2, gamma, beta)
    torch.cuda.synchronize()
    assert torch.equal(mr1, mr2)
    assert torch.equal(g1, g2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,T", [(3, 256), (2, 128), (1, 384)])
def test_gnadd_with_in_launch_statistics(dtype, B, T, tile):
    """Encoder residual block (layers.py:139-178): the 1x1 skip GEMM's GNADD
    epilogue with the GroupNorm statistics merged from the k3 GEMM's GNSTATS
    tiles inside its own launch = vqx_gn_finalize_tiles + GNADD, bit for bit,
    including the mean/rstd it stores for the backward."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    torch.manual_seed(13)
    C = 512
    a = torch.randn(B * T, C, device=DEV).to(dtype)
    c = torch.randn(B * T, C, device=DEV).to(dtype)
    w3 = (torch.randn(C, 3 * C, device=DEV) / (3 * C) ** 0.5).to(dtype)
    w1 = (torch.randn(C, C, device=DEV) / C ** 0.5).to(dtype)
    b3, b1 = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    gamma, beta = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    h = torch.empty(B * T, C, device=DEV, dtype=dtype)
    tiles = torch.empty(B * T // 128 * (C // 128) * 4, device=DEV)
    ops.conv_fwd(a, w3, h, T=T, cin=C, cout=C, ntaps=3, pad=1, bias=b3, gn_stats=tiles, gn_groups=1)
    outs = []
    for fused in (False, True):
        mr = torch.full((B, 1, 2), float("nan"), device=DEV)
        y, y2 = torch.empty(B * T, C, device=DEV, dtype=dtype), torch.empty(B * T, C, device=DEV, dtype=dtype)
        kw = dict(gn_tiles=tiles) if fused else {}
        if not fused:
            ops.gn_finalize_tiles(tiles, B * T, T, C, 1, mr)
        ops.conv_fwd(c, w1, y, T=T, cin=C, cout=C, ntaps=1, pad=0, bias=b1, gn_h=h, gn_mr=mr, gn_gamma=gamma,
                     gn_beta=beta, act=L.PRO_LRELU, y2=y2, **kw)
        torch.cuda.synchronize()
        outs.append((mr, y, y2))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


@pytest.mark.parametrize("n", [4096 * 3 + 4, 1001, 4099, 257])
def test_adam_step_vector_and_scalar_paths_track_torch(n):
    """vqx_grad_sq_norm + vqx_adam_hyper + vqx_adam_step (clip, Adam, StepLR;
    trainer/basic.py:63-75) over three steps (every step clips): the 16-B path
    (16-B aligned buffers; its scalar tail when n % 4 != 0) against the scalar
    path (the same buffers offset by one float) and both against
    torch.optim.Adam (single-tensor, CPU fp32) fed the same clipped gradient,
    to 1e-6 relative.  The two paths are bit-identical (contract(off) honoured
    under -ffp-contract=fast-honor-pragmas; under plain "fast" the packed path
    carried v_pk_fma_f32 and differed by an ulp on half of the second
    moments, tools/adam_dbg.py)."""
    ops = _ops()
    torch.manual_seed(41)
    lr, betas, eps, max_norm = 2e-4, (0.5, 0.999), 1e-8, 1.0
    p0 = torch.randn(n)
    pc = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pc], lr=lr, betas=betas, eps=eps, foreach=False)
    runs = []
    for off in (0, 1):
        base = {k: torch.zeros(n + 4, device=DEV) for k in ("p", "g", "m", "v")}
        runs.append(dict({k: t[off:off + n] for k, t in base.items()},
                         step=torch.zeros(1, dtype=torch.int64, device=DEV), hyper=torch.zeros(16, device=DEV),
                         part=torch.zeros(2048, device=DEV), sumsq=torch.zeros(1, device=DEV)))
        runs[-1]["p"].copy_(p0.to(DEV))
    for s in range(3):
        gs = torch.randn(n) * (3.0 if s == 1 else 0.01)
        for r in runs:
            r["g"].copy_(gs.to(DEV))
        # one clip norm for both (the norm's own summation order follows the buffer's alignment)
        ops.grad_sq_norm(runs[0]["g"], runs[0]["part"], runs[0]["sumsq"])
        for r in runs:
            ops.adam_hyper(r["step"], lr, 1.0, 10 ** 9, betas[0], betas[1], eps, r["hyper"])
            ops.adam_step(r["p"], r["g"], r["m"], r["v"], r["hyper"], runs[0]["sumsq"], max_norm)
        torch.cuda.synchronize()
        for k in ("p", "m", "v"):
            assert torch.equal(runs[0][k], runs[1][k]), (s, k)
        tn = runs[0]["sumsq"].cpu().sqrt()
        coef = (torch.tensor(max_norm) / (tn + 1e-6)).clamp(max=1.0)
        pc.grad = gs * coef
        opt.step()
        st = opt.state[pc]
        assert relerr(runs[0]["p"], pc.detach()) < 1e-6, s
        assert relerr(runs[0]["m"], st["exp_avg"]) < 1e-6 and relerr(runs[0]["v"], st["exp_avg_sq"]) < 1e-6, s


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,C,ld", [(16384, 80, 80), (16384, 64, 64), (16384, 512, 512), (5, 80, 80),
                                    (1000, 7, 7), (4099, 1000, 1000), (777, 128, 192), (65, 8, 8)])
def test_colsum_matches_fp64_and_accumulates(dtype, n, C, ld):
    """vqx_colsum (bias gradients): the narrow-column vector path (lane groups
    narrower than 32), the scalar path (C or ldx not a multiple of the vector
    width), the small-row path, and accumulate=1."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(n + C)
    x = torch.randn(n, ld, generator=g).to(DEV, dtype)
    part = torch.empty(64 * C, device=DEV)
    out = torch.full((C,), 0.5, device=DEV)
    ops.colsum(x, part, out, C=C)
    ref = x[:, :C].double().sum(0)
    tol = 1e-5 * (n ** 0.5) + 1e-5
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=tol)
    ops.colsum(x, part, out, accumulate=True, C=C)
    torch.testing.assert_close(out.double(), 2 * ref, rtol=1e-5, atol=2 * tol)


@pytest.mark.parametrize("B,n_rows", [(64, 100), (64, 3), (5, 40)])
def test_embedding_bwd_rows(B, n_rows):
    """vqx_embedding_bwd_rows (ABI 126): every row of the dense gradient
    written (ids absent from the batch give 0, no zero fill before it), equal
    to zero fill + vqx_embedding_bwd bit for bit (batch-order sums), and
    accumulate = 1 adds."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(B + n_rows)
    D = 128
    dout = torch.randn(B, D, generator=g).to(DEV)
    ids = torch.randint(0, n_rows, (B,), generator=g).to(DEV)
    ref = torch.zeros(n_rows, D, device=DEV)
    ops.embedding_bwd(dout, ids, ref)
    got = torch.full((n_rows, D), float("nan"), device=DEV)
    ops.embedding_bwd_rows(dout, ids, got)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    ops.embedding_bwd_rows(dout, ids, got, accumulate=True)
    torch.cuda.synchronize()
    assert torch.equal(got, ref + ref)


@pytest.mark.parametrize("B,n_rows", [(2500, 7), (1025, 300)])
def test_embedding_bwd_rows_above_one_lds_chunk(B, n_rows):
    """Round 6: batches above the kernel's 1024 staged ids run in
    LDS-sized chunks instead of being refused; each row = its ids' dout rows
    summed (float64 reference, fp32 rounding bar)."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(B)
    D = 128
    dout = torch.randn(B, D, generator=g)
    ids = torch.randint(0, n_rows, (B,), generator=g)
    ref = torch.zeros(n_rows, D, dtype=torch.float64).index_add_(0, ids, dout.double())
    got = torch.full((n_rows, D), float("nan"), device=DEV)
    ops.embedding_bwd_rows(dout.to(DEV), ids.to(DEV), got)
    torch.cuda.synchronize()
    torch.testing.assert_close(got.double().cpu(), ref, rtol=1e-5, atol=1e-4)


def test_guard_canaries_catch_an_out_of_extent_write():
    """vae_npvc_amd/debug.py: a kernel writing one row past a guarded buffer is
    reported by the post-call check with the entry point and the buffer (host
    extent checks off, so the write reaches the device), and a write inside
    the buffer passes."""
    from vae_npvc_amd import debug
    ops = _ops()
    gs = debug.GuardSet(DEV)
    buf = gs.empty(64, 32, dtype=torch.float32, label="probe buffer")
    other = gs.zeros(16, dtype=torch.float32, label="neighbour")
    debug.install(gs)
    try:
        ops.zero_(buf)  # inside: passes the check
        assert gs.checks >= 1
        over = torch.as_strided(buf, (65, 32), (32, 1))  # one row into the tail guard
        ops.set_debug_checks(False)
        with pytest.raises(AssertionError, match=r"vqx_convert_2d.*probe buffer \(tail guard: 128 bytes"):
            ops.convert_2d(None, over)
        assert torch.equal(other.cpu(), torch.zeros(16))
    finally:
        debug.uninstall(gs)
    assert not ops._debug


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,T,ldx", [(64, 80, 256, 80), (3, 80, 100, 128), (2, 7, 33, 7), (1, 80, 1, 80)])
def test_logloss_matches_torch(dtype, B, C, T, ldx):
    """vqx_logloss_fwd_bwd (log_loss, layers.py:283-296): the loss sum and
    dL/dxhat = (xhat - x) * grad_scale, on the 64-frame LDS-tile path (C % 4
    == 0, padded dxhat rows, ragged last tile) and the flat path (C = 7)."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(B * C + T)
    x = torch.randn(B, C, T, generator=g).to(DEV)
    xh_full = torch.randn(B * T, ldx, generator=g).to(DEV)
    xh = xh_full[:, :C]
    dx_full = torch.full((B * T, ldx), 7.0, device=DEV, dtype=dtype)
    dx = dx_full[:, :C]
    loss = torch.zeros(1, device=DEV)
    part = torch.empty(1024, device=DEV)
    gs = 1.0 / (B * T)
    ops.logloss_fwd_bwd(x, xh, gs, dx, loss, part)
    torch.cuda.synchronize()
    d = xh.double().cpu() - x.double().cpu().transpose(1, 2).reshape(B * T, C)
    want = (0.5 * (np.log(2 * np.pi) + d * d)).sum() / (B * T)
    assert abs(loss.item() - want.item()) <= 1e-5 * abs(want.item())
    d32 = xh.cpu() - x.cpu().transpose(1, 2).reshape(B * T, C)  # the kernel's f32 difference and scaling
    torch.testing.assert_close(dx.float().cpu(), (d32 * torch.tensor(gs, dtype=torch.float32)).to(dtype).float(),
                               rtol=0, atol=0)
    if ldx > C:
        assert (dx_full[:, C:] == 7.0).all()  # padding columns untouched


def test_logloss_x_sums_the_vq_partials_like_the_vq_kernel():
    """vqx_logloss_fwd_bwd_x (ABI 126) = vqx_logloss_fwd_bwd plus, in its final
    launch, the VQ commitment sum that vqx_vq_forward computes itself with
    sqerr_out set, bit for bit."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(5)
    N, D, K = 16384, 128, 512
    z = torch.randn(N, D, generator=g).to(DEV)
    E = torch.randn(K, D, generator=g).to(DEV)
    idx = torch.empty(N, dtype=torch.int64, device=DEV)
    part = torch.empty(ops.vq_workspace(N, K, False), device=DEV)
    sq_ref = torch.zeros(1, device=DEV)
    ops.vq_forward(z, E, idx, None, None, sq_ref, part)
    B, C, T = 64, 80, 256
    x = torch.randn(B, C, T, generator=g).to(DEV)
    xh = torch.randn(B * T, C, generator=g).to(DEV)
    dx1, dx2 = (torch.empty(B * T, C, device=DEV, dtype=torch.bfloat16) for _ in range(2))
    l1, l2, sq = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    lp = torch.empty(1024, device=DEV)
    ops.logloss_fwd_bwd(x, xh, 1.0 / (B * T), dx1, l1, lp)
    n = (N + ops.VQ_FRAMES - 1) // ops.VQ_FRAMES
    ops.logloss_fwd_bwd_x(x, xh, 1.0 / (B * T), dx2, l2, lp, part[:n], sq)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(dx1, dx2) and torch.equal(sq, sq_ref)


def test_ema_update_clear_equals_update_and_zeroes_the_statistics():
    """vqx_vq_ema_update_clear (ABI 126) = vqx_vq_ema_update bit for bit
    (codebook, EMA buffers, diagnostics), with bsum / bcnt zero afterwards."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(21)
    K, D = 512, 128
    base = dict(emb_sum=torch.randn(K, D, generator=g), emb_elem=torch.rand(K, generator=g) * 3,
                E=torch.randn(K, D, generator=g), bsum=torch.randn(K, D, generator=g),
                bcnt=torch.randint(0, 5, (K,), generator=g).float(), rand=torch.randn(K, D, generator=g))
    res = []
    for clear in (False, True):
        t = {k: v.clone().to(DEV) for k, v in base.items()}
        diag = torch.zeros(4, device=DEV)
        ops.vq_ema_update(t["emb_sum"], t["emb_elem"], t["E"], t["bsum"], t["bcnt"], t["rand"], 0.99, 1.0, diag,
                          clear=clear)
        torch.cuda.synchronize()
        res.append((t, diag))
    (a, da), (b, db) = res
    for k in ("emb_sum", "emb_elem", "E"):
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(da, db)
    assert torch.equal(a["bsum"], base["bsum"].to(DEV)) and torch.equal(a["bcnt"], base["bcnt"].to(DEV))
    assert not b["bsum"].any() and not b["bcnt"].any()


def test_sq_norm_finish_adam_equals_finish_then_hyper():
    """vqx_sq_norm_finish_adam (ABI 126) = vqx_sq_norm_finish + vqx_adam_hyper,
    bit for bit: the norm, the per-step scalars (StepLR decay at step 4) and the
    step counter, advanced once per call."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(12)
    part = torch.randn(110_000, generator=g).abs().to(DEV)
    flat = torch.randn(300_000, generator=g).to(DEV)
    rng = torch.tensor([[1000, 5000], [200_000, 70_000]], dtype=torch.int64).to(DEV)
    outs = []
    for fused in (False, True):
        step = torch.zeros(1, dtype=torch.int64, device=DEV)
        hyper = torch.zeros(16, device=DEV)
        out, scratch = torch.zeros(1, device=DEV), torch.zeros(256, device=DEV)
        hist = []
        for _ in range(5):
            if fused:
                ops.sq_norm_finish_adam(part, flat, rng, out, scratch, step, 2e-4, 0.5, 4, 0.9, 0.999, 1e-8, hyper)
            else:
                ops.sq_norm_finish(part, flat, rng, out, scratch)
                ops.adam_hyper(step, 2e-4, 0.5, 4, 0.9, 0.999, 1e-8, hyper)
            hist.append((out.clone(), hyper.clone(), step.clone()))
        torch.cuda.synchronize()
        outs.append(hist)
    for (o1, h1, s1), (o2, h2, s2) in zip(*outs):
        assert torch.equal(o1, o2) and torch.equal(h1, h2) and torch.equal(s1, s2)
    assert int(outs[1][-1][2]) == 5


@pytest.mark.parametrize("B", [64, 13])
def test_linear_cond_ids_equal_lookup_then_linear(B):
    """vqx_linear_batched_fwd_ids / _bwd_ids (ABI 126: rows of the embedding
    table read in the operand loads) = vqx_embedding_fwd + the plain batched
    calls, bit for bit (the same kernels on the same rows)."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(40 + B)
    n, I, O, n_spk = 10, 128, 1024, 100
    emb = torch.randn(n_spk, I, generator=g).to(DEV)
    ids = torch.randint(0, n_spk, (B,), generator=g).to(DEV)
    runs = []
    for use_ids in (False, True):
        gg = torch.Generator(device="cpu").manual_seed(3)
        lay = [dict(W=(torch.randn(O, I, generator=gg) / I ** 0.5).to(DEV), bias=torch.randn(O, generator=gg).to(DEV),
                    out=torch.empty(B, O, device=DEV), dout=torch.randn(B, O, generator=gg).to(DEV),
                    dW=torch.empty(O, I, device=DEV), dbias=torch.empty(O, device=DEV)) for _ in range(n)]
        tab = ops.linear_table(lay)
        dc = torch.empty(B, I, device=DEV)
        part = torch.empty(n * (O // 64) * B * I, device=DEV)
        if use_ids:
            assert ops.linear_ids_ok(B, I, O, emb)
            ops.linear_batched_fwd_ids(tab, emb, ids, B, I, O)
            ops.linear_batched_bwd_ids(tab, emb, ids, B, I, O, dc, part)
        else:
            c = torch.empty(B, I, device=DEV)
            ops.embedding_fwd(emb, ids, c)
            ops.linear_batched_fwd(tab, c, B, I, O)
            ops.linear_batched_bwd(tab, c, B, I, O, dc, part)
        torch.cuda.synchronize()
        runs.append((lay, dc))
    (la, dca), (lb, dcb) = runs
    for a, b in zip(la, lb):
        for k in ("out", "dW", "dbias"):
            assert torch.equal(a[k], b[k]), k
    assert torch.equal(dca, dcb)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,C,ld", [(16384, 80, 80), (16384, 128, 128), (777, 128, 192), (65, 8, 8), (5, 80, 80)])
def test_colsum_partials_sum_to_colsum(dtype, n, C, ld):
    """vqx_colsum_partials (ABI 126: the first level alone, for a bias gradient
    reduced by the weight-norm backward's column reduce) equals vqx_colsum's
    two levels up to summation order."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(n + 3 * C)
    x = torch.randn(n, ld, generator=g).to(DEV, dtype)[:, :C]
    npart = ops.colsum_parts(n, C, dtype)
    assert 1 <= npart <= 64
    part = torch.empty(npart, C, device=DEV)
    ops.colsum_partials(x, part)
    ref = x.double().sum(0)
    tol = 1e-5 * (n ** 0.5) + 1e-5
    torch.testing.assert_close(part.double().sum(0), ref, rtol=1e-5, atol=tol)
    with pytest.raises(ValueError):
        ops.colsum_partials(x, torch.empty(npart + 1, C, device=DEV))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,D", [(16384, 128), (16384, 64), (1000, 256), (100, 128)])
def test_commit_bwd_with_column_sums(dtype, N, D):
    """vqx_vq_commit_bwd_cs writes the same dz as vqx_vq_commit_bwd, bit for
    bit, and per row part the column sums of the stored dz (the encoder output
    conv's bias gradient); parts past N rows (N < 256) are zero."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(N + D)
    z, zq = (torch.randn(N, D, generator=g).to(DEV) for _ in range(2))
    scale = 2.0 * 0.25 / N
    dz1 = torch.empty(N, D, device=DEV, dtype=dtype)
    dz2 = torch.empty_like(dz1)
    part = torch.full((ops.COMMIT_PARTS, D), float("nan"), device=DEV)
    ops.vq_commit_bwd(z, zq, scale, dz1)
    ops.vq_commit_bwd_cs(z, zq, scale, dz2, part)
    torch.cuda.synchronize()
    assert torch.equal(dz1, dz2)
    assert torch.isfinite(part).all()
    P = ops.COMMIT_PARTS
    for p in (0, P // 2, P - 1):
        r0, r1 = N * p // P, N * (p + 1) // P
        ref = dz1[r0:r1].double().sum(0)
        torch.testing.assert_close(part[p].double(), ref, rtol=1e-5, atol=1e-6 * scale * max(1, r1 - r0))
    torch.testing.assert_close(part.double().sum(0), dz1.double().sum(0), rtol=1e-5, atol=1e-5 * scale * N ** 0.5)


@pytest.mark.parametrize("K,N", [(512, 16384), (1024, 300), (7, 5)])
def test_gather_rows_host_indices_equal_device_indices(K, N):
    """vqx_gather_rows_host (row ids in host memory, passed to the kernels by
    value, 512 a launch) writes exactly what vqx_gather_rows does with the
    same ids on the device, including -1 (zero rows: another rank's frames)
    and K above one launch's 512 rows."""
    from vae_npvc_amd import ops
    g = torch.Generator().manual_seed(K + N)
    D = 128
    src = torch.randn(N, D, generator=g).cuda()
    rows = torch.randint(-1, N, (K,), generator=g)
    a = torch.full((K, D), 7.0, device="cuda")
    b = torch.full((K, D), 9.0, device="cuda")
    ops.gather_rows(src, rows.cuda(), a)
    ops.gather_rows_host(src, rows.to(torch.int32), b)
    assert torch.equal(a, b)
    ref = torch.where((rows >= 0)[:, None], src.cpu()[rows.clamp_min(0)], torch.zeros(1))
    assert torch.equal(b.cpu(), ref)


@pytest.mark.parametrize("r,c,shift,splits,B,T", [(512, 512, 1, 8, 8, 256), (512, 1024, -1, 4, 8, 256),
                                                  (256, 512, 1, 5, 3, 128), (128, 64, -1, 3, 2, 64),
                                                  (256, 128, 1, 6, 4, 128), (128, 256, -1, 7, 2, 256)])
def test_wgrad_in_launch_split_k_reduction(r, c, shift, splits, B, T):
    """vqx_wgrad_args.fixup_dw (ABI 127): the last split of each tile sums the
    bf16 slabs of its tile in split order in fp32 inside the launch.  fixup_dw
    equals that sum formed from the slabs afterwards (acc = 0, acc += slab s:
    the weight-norm backward's order) bit for bit; the slabs equal those of a
    call without the reduction; the tile counters are left zero, so a second
    call (and the fused DGRAD + WGRAD launch) gives the same bits."""
    ops = _ops()
    from vae_npvc_amd import _lib as L
    g = torch.Generator(device="cpu").manual_seed(r + c + splits)
    N = B * T
    p = torch.randn(N, r, generator=g).to(DEV, torch.bfloat16)
    q = torch.randn(N, c, generator=g).to(DEV, torch.bfloat16)
    assert ops.wgrad_fixup_ok(N, T, r, c, 3, 1, L.VQX_BF16, L.VQX_BF16)
    assert not ops.wgrad_fixup_ok(N, T, r, c, 3, 1, L.VQX_BF16, L.VQX_F32)
    kw = dict(T=T, r_dim=r, c_dim=c, ntaps=3, pad=1, shift_sign=shift, splits=splits)
    ref_slabs = torch.empty(splits, r, 3 * c, device=DEV, dtype=torch.bfloat16)
    ops.conv_wgrad(p, q, ref_slabs, **kw)
    # the weight-norm backward's order (vqx_misc.hip wn_bwd_kernel, 256-thread blocks): one
    # sequential sum for rows of >= 256 four-column groups, else G interleaved split groups
    nx4 = 3 * c // 4
    G = 1 if nx4 >= 256 else min(splits, 256 // nx4)
    acc = torch.zeros(r, 3 * c, device=DEV)
    for gi in range(G):
        part = torch.zeros(r, 3 * c, device=DEV)
        for s in range(gi, splits, G):
            part += ref_slabs[s].float()
        acc += part
    cnt = torch.zeros(((r + 127) // 128) * (c // 64 + 1), device=DEV, dtype=torch.int32)
    for it in range(2):
        slabs = torch.full((splits, r, 3 * c), float("nan"), device=DEV, dtype=torch.bfloat16)
        dw = torch.full((r, 3 * c), float("nan"), device=DEV)
        ops.conv_wgrad(p, q, slabs, fixup_dw=dw, fixup_counters=cnt, **kw)
        torch.cuda.synchronize()
        assert torch.equal(slabs, ref_slabs), it
        assert torch.equal(dw, acc), (it, float((dw - acc).abs().max()))
        assert int(cnt.abs().sum()) == 0
    # the fused DGRAD + WGRAD launch (3-tap interleaved kernel) takes the same path
    if shift == 1:
        wt = (torch.randn(r, c, 3, generator=g) / (3 * c) ** 0.5).to(DEV, torch.bfloat16)
        dx = torch.empty(N, c, device=DEV, dtype=torch.bfloat16)
        dw2 = torch.full((r, 3 * c), float("nan"), device=DEV)
        fused = ops.conv_dgrad_wgrad(p, pack(wt), dx, dict(T=T, cin=r, cout=c, ntaps=3, pad=1), p, q, slabs,
                                     dict(kw, fixup_dw=dw2, fixup_counters=cnt))
        torch.cuda.synchronize()
        assert torch.equal(dw2, acc) and int(cnt.abs().sum()) == 0, fused


def test_host_mailbox_publishes_in_stream_order():
    """vqx_mailbox_* (ABI 127): values published on the stream arrive in the
    host slot with the step's sequence number, behind earlier work on the same
    stream; a slot reused by a later publish reports LookupError (the reader
    then takes the device copy); many publishes in flight keep their order."""
    ops = _ops()
    mb = ops.Mailbox(slots=4, floats=16)
    x = torch.arange(8, device=DEV, dtype=torch.float32)
    big = torch.randn(4096, 4096, device=DEV)
    for _ in range(3):  # queue some work ahead of the publish
        big = big @ big.t() * 1e-3
    copy = torch.empty(8, device=DEV)
    seq, slot = mb.publish(x + big[0, 0] * 0, copy)
    got = None
    for _ in range(10_000_000):
        got = mb.try_read(seq, slot, 8)
        if got is not None:
            break
    assert got is not None and np.array_equal(got, np.arange(8, dtype=np.float32)), got
    torch.cuda.synchronize()
    assert torch.equal(copy, x)
    pubs = [mb.publish(x + k) for k in range(6)]  # slots wrap: the first two are reused
    torch.cuda.synchronize()
    with pytest.raises(LookupError):
        mb.try_read(*pubs[0], 8)
    for k in (4, 5):
        s, sl = pubs[k]
        assert np.array_equal(mb.try_read(s, sl, 8), np.arange(8, dtype=np.float32) + k)


@pytest.mark.parametrize("jobs", ["all", "wn", "cond", "x", "cond+x"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_step_prologue_equals_the_three_launches(jobs, dtype):
    """vqx_step_prologue (ABI 128: ConvT packs + conditioning linears + input
    transpose in one grid) = vqx_weight_norm_fwd_flags(NORMS_READY) +
    vqx_linear_batched_fwd_ids + vqx_nct_to_ntc, bit for bit, for any subset
    of the jobs (mixed-kind pack table, ragged transpose tiles, B < 16)."""
    ops = _ops()
    specs = [(1, 512, 1024, 3), (1, 100, 70, 3), (0, 512, 640, 1), (0, 96, 80, 5), (1, 64, 48, 5)]
    B, I, O, n, n_spk, C, T = 13, 128, 1024, 7, 50, 80, 200
    runs = []
    for fused in (False, True):
        g = torch.Generator(device="cpu").manual_seed(77)
        ents = []
        for kind, cin, cout, k in specs:
            shape = (cout, cin, k) if kind == 0 else (cin, cout, k)
            v = torch.randn(*shape, generator=g).to(DEV)
            rows = shape[0]
            ents.append(dict(v=v, g=(torch.rand(rows, generator=g) + 0.5).to(DEV),
                             w_packed=torch.zeros(cout, k * cin, device=DEV, dtype=dtype),
                             norm=torch.zeros(rows, device=DEV), kind=kind, cout=cout, cin=cin, k=k,
                             dtype=ops.dt_code(dtype)))
        wt = ops.wn_table(ents)
        ops.weight_norm_fwd(wt)  # the row norms current (what vqx_adam_step_wn leaves)
        for e in ents:
            e["w_packed"].zero_()
        emb = torch.randn(n_spk, I, generator=g).to(DEV)
        ids = torch.randint(0, n_spk, (B,), generator=g).to(DEV)
        lay = [dict(W=(torch.randn(O, I, generator=g) / I ** 0.5).to(DEV), bias=torch.randn(O, generator=g).to(DEV),
                    out=torch.zeros(B, O, device=DEV), dout=torch.zeros(B, O, device=DEV),
                    dW=torch.zeros(O, I, device=DEV), dbias=torch.zeros(O, device=DEV)) for _ in range(n)]
        tab = ops.linear_table(lay)
        x = torch.randn(B, C, T, generator=g).to(DEV)
        y = torch.zeros(B * T, 96, device=DEV, dtype=dtype)  # ld > C
        do_wn, do_c, do_x = jobs in ("all", "wn"), jobs in ("all", "cond", "cond+x"), jobs in ("all", "x", "cond+x")
        if fused:
            ops.step_prologue(wt if do_wn else None, (tab, emb, ids, B, I, O) if do_c else None,
                              x if do_x else None, y if do_x else None)
        else:
            if do_wn:
                ops.weight_norm_fwd(wt, flags=ops.WNF_NORMS_READY)
            if do_c:
                ops.linear_batched_fwd_ids(tab, emb, ids, B, I, O)
            if do_x:
                ops.nct_to_ntc(x, y)
        torch.cuda.synchronize()
        runs.append(([e["w_packed"] for e in ents] + [e["norm"] for e in ents] + [l_["out"] for l_ in lay], y))
    (ta, ya), (tb, yb) = runs
    for a, b in zip(ta, tb):
        assert torch.equal(a, b)
    assert torch.equal(ya, yb)
    if jobs in ("all", "x", "cond+x"):
        assert bool(ya.abs().sum() > 0)


@pytest.mark.parametrize("n_vq,rows", [(0, False), (512, False), (512, True)])
def test_ema_update_close_equals_the_separate_launches(n_vq, rows):
    """vqx_vq_ema_update_close (ABI 128) = vqx_logloss_fwd_bwd(_x)'s sums +
    vqx_vq_ema_update_clear + vqx_mailbox_publish, bit for bit: the loss and
    commitment sums, codebook, EMA buffers, diagnostics (the 1024-thread sums
    formed by four virtual threads per thread) and the published values, with
    the arrival counter left zero for the next call; rows: the dead-code rows
    read from z inside the launch = vqx_gather_rows_host first (negative
    indices: zero rows)."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(23)
    K, D, B, C, T = 512, 64, 8, 80, 200
    base = dict(emb_sum=torch.randn(K, D, generator=g), emb_elem=torch.rand(K, generator=g) * 3,
                E=torch.randn(K, D, generator=g), bsum=torch.randn(K, D, generator=g),
                bcnt=torch.randint(0, 5, (K,), generator=g).float(), rand=torch.randn(K, D, generator=g))
    x = torch.randn(B, C, T, generator=g).to(DEV)
    xhat = torch.randn(B * T, C, generator=g).to(DEV)
    vq_part = torch.rand(max(n_vq, 1), generator=g).to(DEV)
    z = torch.randn(3000, D, generator=g).to(DEV)
    perm = torch.randperm(3000, generator=g)[:K].to(torch.int32)
    perm[::7] = -1
    mb = ops.Mailbox(slots=4, floats=16)
    res = []
    for fused in (False, True):
        t = {k: v.clone().to(DEV) for k, v in base.items()}
        stats = torch.zeros(8, device=DEV)
        dx = torch.empty(B * T, C, device=DEV)
        lp = torch.zeros(1024, device=DEV)
        part = torch.zeros(ops.ema_workspace(K, D), device=DEV)
        copy = torch.zeros(8, device=DEV)
        for rep in range(2):  # the second call checks the counter was left zero
            t["bsum"].copy_(base["bsum"])  # (the first call cleared them)
            t["bcnt"].copy_(base["bcnt"])
            if fused:
                n = ops.logloss_parts(x, xhat, 1.0 / (B * T), dx, lp)
                sums = [(lp[:n], float(np.float32(1.0) / (np.float32(B) * np.float32(T))), stats[0:1])]
                if n_vq:
                    sums.append((vq_part[:n_vq], 1.0, stats[1:2]))
                seq, slot = ops.vq_ema_update(t["emb_sum"], t["emb_elem"], t["E"], t["bsum"], t["bcnt"], t["rand"],
                                              0.99, 1.0, stats[4:8], part, clear=True, sums=sums,
                                              publish=(mb, stats, copy), rows=(z, perm) if rows else None)
            else:
                if n_vq:
                    ops.logloss_fwd_bwd_x(x, xhat, 1.0 / (B * T), dx, stats[0:1], lp, vq_part[:n_vq], stats[1:2])
                else:
                    ops.logloss_fwd_bwd(x, xhat, 1.0 / (B * T), dx, stats[0:1], lp)
                if rows:
                    ops.gather_rows_host(z, perm, t["rand"])
                ops.vq_ema_update(t["emb_sum"], t["emb_elem"], t["E"], t["bsum"], t["bcnt"], t["rand"], 0.99, 1.0,
                                  stats[4:8], part, clear=True)
                seq, slot = mb.publish(stats, copy)
        torch.cuda.synchronize()
        got = None
        for _ in range(1_000_000):
            got = mb.try_read(seq, slot, 8)
            if got is not None:
                break
        res.append((t, stats.clone(), copy.clone(), got, part[-1].item()))
    (a, sa, ca, ga, za), (b, sb, cb, gb, zb) = res
    for k in ("emb_sum", "emb_elem", "E", "bsum", "bcnt"):
        assert torch.equal(a[k], b[k]), k
    assert torch.equal(sa, sb), (sa, sb)
    assert torch.equal(ca, cb) and torch.equal(cb, sb)
    assert np.array_equal(ga, gb) and np.array_equal(gb, sb.cpu().numpy())
    assert za == 0.0 and zb == 0.0
