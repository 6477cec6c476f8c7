"""Resampling convolutions of the multi-resolution models:
the weight-normed strided Conv1d that down-samples by `scale` (vqvae.py:144-156,
vqvae2.py:197-226: kernel 2s, stride s, padding s//2 + s%2) and the
ConvTranspose1d that up-samples (vqvae.py:243-263, vqvae2.py:297-319: same
kernel / padding, output_padding s%2), on the MI355X.

No new GEMM: folding s consecutive frames into channels (a free
reinterpretation of the frame-major [N, C] layout as [N/s, s*C]) turns the
strided conv into a stride-1, 3-tap, pad-1 conv whose packed weight the
weight-norm kernel writes directly (include/vqx.h VQX_WN_RESAMPLE).  So:

  down-sampling Conv1d    fwd = vqx_conv1d_fwd   on the folded input,
                          dx  = vqx_conv1d_dgrad (folded output = dx),
                          dW  = vqx_conv1d_wgrad -> weight-norm backward;
  up-sampling ConvT       fwd = vqx_conv1d_dgrad (its adjoint), dx = fwd,
                          dW  = vqx_conv1d_wgrad with the roles swapped.

The folded 3-tap form multiplies by one structurally zero tap in three
(k = 2s of 3s slots): 1.5x the algorithmic FLOPs, in exchange for running
on the same MFMA kernels and layouts as the rest of the step.

Parameters and state_dict keys are the reference's (`bias`, `weight_g`,
`weight_v` from nn.utils.weight_norm, dim 0).  Inputs are (B, C, T) like the
reference modules; T must be a multiple of `scale` for the down-sampler.
"""
import math

import torch
import torch.nn as nn

from .. import _lib as L
from .. import ops

F32 = torch.float32


def resample_geometry(scale):
    """(kernel, padding, output_padding) of vqvae.py:150-156 / 247-254."""
    if scale < 2:
        raise ValueError("a resampling conv has scale >= 2 (scale 1 is the stride-1 conv)")
    return 2 * scale, scale // 2 + scale % 2, scale % 2


class ResampleConv1d(nn.Module):
    """Weight-normed Conv1d(cin, cout, 2s, stride=s) (transposed=False) or
    ConvTranspose1d(cin, cout, 2s, stride=s, output_padding=s%2)
    (transposed=True), computed by libvqx."""

    def __init__(self, cin, cout, scale, transposed=False, compute_dtype="fp32", splits=None, weight_norm=True):
        super().__init__()
        self.cin, self.cout, self.scale, self.transposed = cin, cout, scale, transposed
        self.k, self.padding, self.output_padding = resample_geometry(scale)
        self.cd = torch.bfloat16 if compute_dtype in ("bf16", "bfloat16") else F32
        fan_in = (cout if transposed else cin) * self.k
        bound = 1.0 / math.sqrt(fan_in)
        vshape = (cin, cout, self.k) if transposed else (cout, cin, self.k)
        v = torch.empty(vshape).uniform_(-bound, bound)
        self.splits = splits
        self.has_weight_norm = bool(weight_norm)
        if not weight_norm:  # a plain strided Conv1d / ConvTranspose1d: weight, bias (use_weight_norm: false)
            nn.init.kaiming_normal_(v, nonlinearity="relu")  # reset_parameters, vqvae.py:210-217 (as WNConv1d)
            self.weight = nn.Parameter(v)
            self.bias = nn.Parameter(torch.empty(cout).uniform_(-bound, bound))
            return
        self.bias = nn.Parameter(torch.empty(cout).uniform_(-bound, bound))
        self.weight_g = nn.Parameter(v.flatten(1).norm(dim=1).view(vshape[0], 1, 1))
        self.weight_v = nn.Parameter(v)

    def remove_weight_norm(self):
        """torch.nn.utils.remove_weight_norm (vqvae.py:93-103): bake w = g*v/||v||
        (norm over all dims but 0) into a plain `weight` registered after `bias`."""
        if not self.has_weight_norm:
            raise ValueError("weight_norm not present")
        w = torch._weight_norm(self.weight_v, self.weight_g, 0).detach()
        del self.weight_g
        del self.weight_v
        self.weight = nn.Parameter(w)
        self.has_weight_norm = False

    @property
    def v_param(self):
        """The direction parameter the packing kernel reads: weight_v, or the plain weight."""
        return self.weight_v if self.has_weight_norm else self.weight

    @property
    def g_param(self):
        return self.weight_g if self.has_weight_norm else None

    @property
    def rows(self):
        return self.cin if self.transposed else self.cout

    @property
    def fold_c(self):  # channels folded per tap group
        return self.cout if self.transposed else self.cin

    def extra_repr(self):
        return (f"{self.cin}, {self.cout}, kernel_size={self.k}, stride={self.scale}, padding={self.padding}, "
                f"transposed={self.transposed}")

    def _table(self, w_packed, norm, dv=None, dg=None, slabs=None, splits=1):
        kind = L.WN_RESAMPLE_T if self.transposed else L.WN_RESAMPLE
        return ops.wn_table([dict(v=self.v_param, g=self.g_param, w_packed=w_packed, norm=norm, dv=dv, dg=dg,
                                  slabs=slabs, kind=kind, cout=self.cout, cin=self.cin, k=self.k, splits=splits,
                                  dtype=ops.dt_code(w_packed.dtype), stride=self.scale, pad=self.padding)])

    def forward(self, x):
        if not self.has_weight_norm:
            return _ResampleFn.apply(self, x, self.bias, None, self.weight)
        return _ResampleFn.apply(self, x, self.bias, self.weight_g, self.weight_v)


class _ResampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, bias, g, v):
        if not x.is_cuda:
            raise L.VqxError("ResampleConv1d runs on the MI355X only (libvqx); move it with .cuda()")
        B, C, T = x.shape
        s, cd, dev = mod.scale, mod.cd, x.device
        if C != mod.cin:
            raise ValueError(f"ResampleConv1d: input has {C} channels, the layer takes {mod.cin}")
        R, FC = mod.rows, mod.fold_c
        wp = torch.empty(R, 3 * s * FC, device=dev, dtype=cd)
        norm = torch.empty(R, device=dev, dtype=F32)
        ops.weight_norm_fwd(mod._table(wp, norm))
        xr = torch.empty(B * T, C, device=dev, dtype=cd)
        ops.nct_to_ntc(x.float().contiguous(), xr)
        if not mod.transposed:  # down-sample: T/s output frames
            if T % s:
                raise ValueError(f"ResampleConv1d: T={T} is not a multiple of the scale {s}")
            To = T // s
            y = torch.empty(B * To, mod.cout, device=dev, dtype=cd)
            ops.conv_fwd(xr.view(B * To, s * C), wp, y, T=To, cin=s * C, cout=mod.cout, ntaps=3, pad=1, bias=bias)
        else:  # up-sample: s*T output frames, computed folded [B*T, s*cout]
            To = T * s
            y = torch.empty(B * To, mod.cout, device=dev, dtype=cd)
            btile = torch.empty(s, mod.cout, device=dev, dtype=F32)
            ops.convert_2d(bias.detach().view(1, -1).expand(s, -1), btile)
            ops.conv_dgrad(xr, wp, y.view(B * T, s * mod.cout), T=T, cin=C, cout=s * mod.cout, ntaps=3, pad=1,
                           bias=btile.view(-1))
        out = torch.empty(B, mod.cout, To, device=dev, dtype=F32)
        ops.ntc_to_nct(y, out)
        ctx.mod, ctx.shape = mod, (B, C, T, To)
        ctx.save_for_backward(xr, wp, norm)
        return out

    @staticmethod
    def backward(ctx, gout):
        mod = ctx.mod
        B, C, T, To = ctx.shape
        xr, wp, norm = ctx.saved_tensors
        s, cd, dev = mod.scale, mod.cd, gout.device
        R, FC = mod.rows, mod.fold_c
        dy = torch.empty(B * To, mod.cout, device=dev, dtype=cd)
        ops.nct_to_ntc(gout.float().contiguous(), dy)
        dx = torch.empty(B * T, C, device=dev, dtype=cd)
        n_fold = B * To if not mod.transposed else B * T     # folded GEMM rows
        T_fold = To if not mod.transposed else T
        splits = mod.splits or max(1, min(64, n_fold // 256))
        slabs = torch.empty(splits, R, 3 * s * FC, device=dev, dtype=F32)
        if not mod.transposed:
            ops.conv_dgrad(dy, wp, dx.view(B * To, s * C), T=To, cin=mod.cout, cout=s * C, ntaps=3, pad=1)
            ops.conv_wgrad(dy, xr.view(B * To, s * C), slabs, T=T_fold, r_dim=mod.cout, c_dim=s * C, ntaps=3, pad=1,
                           shift_sign=1, splits=splits)
        else:
            dyf = dy.view(B * T, s * mod.cout)
            ops.conv_fwd(dyf, wp, dx, T=T, cin=s * mod.cout, cout=C, ntaps=3, pad=1)
            ops.conv_wgrad(xr, dyf, slabs, T=T_fold, r_dim=C, c_dim=s * mod.cout, ntaps=3, pad=1, shift_sign=1,
                           splits=splits)
        dv = torch.empty_like(mod.v_param)
        dg = torch.empty_like(mod.weight_g) if mod.has_weight_norm else None
        ops.weight_norm_bwd(mod._table(wp, norm, dv=dv, dg=dg, slabs=slabs, splits=splits))
        part = torch.empty(64 * mod.cout, device=dev, dtype=F32)
        dbias = torch.empty(mod.cout, device=dev, dtype=F32)
        ops.colsum(dy, part, dbias)
        dxo = torch.empty(B, C, T, device=dev, dtype=F32)
        ops.ntc_to_nct(dx, dxo)
        return None, dxo, dbias, dg, dv
