"""Resampling convs (vqvae.py:144-156 / 243-263,
vqvae2.py:197-226 / 297-319) on the MI355X against torch's fp64 CPU
Conv1d / ConvTranspose1d with weight norm: forward, input, bias, g and v
gradients.  fp32 mode within 2e-5 relative, bf16 within 2e-2."""
import pytest
import torch
import torch.nn.functional as F

from vae_npvc_amd.model.resample import ResampleConv1d, resample_geometry

CASES = [  # transposed, scale, cin, cout, B, T
    (False, 2, 64, 128, 2, 128),
    (False, 4, 128, 64, 3, 256),
    (False, 3, 64, 64, 2, 96),
    (True, 2, 128, 64, 2, 64),
    (True, 4, 64, 128, 2, 64),
    (True, 3, 64, 64, 2, 32),
]


def _reference(mod, x, R):
    v = mod.weight_v.detach().double().cpu().requires_grad_()
    g = mod.weight_g.detach().double().cpu().requires_grad_()
    b = mod.bias.detach().double().cpu().requires_grad_()
    xr = x.detach().double().cpu().requires_grad_()
    w = torch._weight_norm(v, g, 0)
    k, p, op = resample_geometry(mod.scale)
    if mod.transposed:
        y = F.conv_transpose1d(xr, w, b, stride=mod.scale, padding=p, output_padding=op)
    else:
        y = F.conv1d(xr, w, b, stride=mod.scale, padding=p)
    (y * R.double().cpu()).sum().backward()
    return y.detach(), xr.grad, b.grad, g.grad, v.grad


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def test_resample_module_keys_match_torch_weight_norm():
    for transposed in (False, True):
        mod = ResampleConv1d(64, 32, 2, transposed=transposed)
        ref = (torch.nn.ConvTranspose1d if transposed else torch.nn.Conv1d)(64, 32, 4, stride=2, padding=1)
        ref = torch.nn.utils.weight_norm(ref)
        assert {k: tuple(v.shape) for k, v in mod.state_dict().items()} == \
            {k: tuple(v.shape) for k, v in ref.state_dict().items()}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("transposed,scale,cin,cout,B,T", CASES)
def test_resample_conv_matches_torch(dtype, transposed, scale, cin, cout, B, T):
    torch.manual_seed(scale * 10 + int(transposed))
    mod = ResampleConv1d(cin, cout, scale, transposed=transposed, compute_dtype=dtype).cuda()
    with torch.no_grad():
        mod.weight_g.mul_(1.5)  # g != ||v||, so the norm's gradient is exercised
    x = torch.randn(B, cin, T, device="cuda", requires_grad=True)
    y = mod(x)
    To = T * scale if transposed else T // scale
    assert y.shape == (B, cout, To)
    R = torch.randn_like(y)
    (y * R).sum().backward()
    yr, dxr, dbr, dgr, dvr = _reference(mod, x, R)
    tol = 2e-5 if dtype == "fp32" else 2e-2
    assert rel(y.detach(), yr) < tol
    assert rel(x.grad, dxr) < tol
    assert rel(mod.bias.grad, dbr) < tol
    assert rel(mod.weight_g.grad, dgr) < tol * 5
    assert rel(mod.weight_v.grad, dvr) < tol * 5
