"""Encoder backward at fp32 precision with an injected, well-conditioned dL/dz
(VERDICT r02 "weak #1").

In the training step the encoder's only gradient is beta * the commitment
term 2(z - z_q)/(B T) (layers_vq.py:301,315), a difference of nearly equal
vectors, so the step-level golden tests can only pin the encoder gradients to
~1e-3.  Here the SAME seeded dL/dz drives both the HIP encoder backward
(engine.encoder_bwd(dz=...): ten GroupNorm backwards, the fused DGRAD+WGRAD
launches, the split-K slabs and the weight-norm backward of every encoder
conv) and torch.autograd of the oracle encoder (vqvae.py:185-192,
layers.py:129-178) evaluated in float64, linearised at the HIP forward's
LeakyReLU sign pattern (a pre-activation within rounding of 0 can take
either slope: with 10 blocks ~1 of 262 K such elements flips and moves a
gradient by ~1e-2).  Every encoder.* gradient must be within 1e-5 of the
float64 truth, elementwise, relative to the tensor's largest entry; the
oracle's own fp32 CPU gradients are reported beside it.
Recipes: vcc20 (config 2 widths), aishell3 (160 mel) and the general
two-stage topology (stride-2 resampling, dilation, stack_layers 2)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

BAR = 1e-5


class _MaskedLeakyReLU(torch.autograd.Function):
    """LeakyReLU(0.2) whose derivative takes the sign pattern from a given
    mask (the HIP forward's own stored LeakyReLU output) instead of from x."""

    @staticmethod
    def forward(ctx, x, mask):
        ctx.save_for_backward(mask)
        return torch.nn.functional.leaky_relu(x, 0.2)

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        return g * torch.where(mask > 0, 1.0, 0.2).to(g.dtype), None


class _FWithMasks:
    """torch.nn.functional for the oracle module, with leaky_relu drawing its
    derivative masks from a queue (in the oracle encoder's call order)."""

    def __init__(self, masks):
        self.masks = list(masks)

    def __getattr__(self, name):
        return getattr(torch.nn.functional, name)

    def leaky_relu(self, x, slope=0.01):
        assert slope == 0.2 and self.masks, "unexpected LeakyReLU call"
        m = self.masks.pop(0)
        assert m.shape == x.shape, (m.shape, x.shape)
        return _MaskedLeakyReLU.apply(x, m.to(x.dtype))


def hip_lrelu_masks(w):
    """The HIP forward's stored LeakyReLU outputs, (B, C, T) each, in the
    order the oracle encoder (oracle/vqvae_cpu.py encoder) applies LeakyReLU:
    per stage the previous stage's output, then per block and stack layer its
    input (a_j for the first layer, LeakyReLU(GN(h)) for the next), and the
    output LeakyReLU before the 1x1 conv to z."""
    B = w.B

    def nct(t, T):
        return t.detach().double().cpu().view(B, T, -1).permute(0, 2, 1)
    out = []
    for si, sw in enumerate(w.enc):
        if si > 0:
            prev = w.enc[si - 1]
            out.append(nct(prev.a[-1], prev.T))
        for j in range(len(sw.h)):
            out.append(nct(sw.a[j], sw.T))
            for l in range(1, len(sw.h[j])):
                out.append(nct(sw.g[j][l - 1], sw.T))
    last = w.enc[-1]
    out.append(nct(last.a[-1], last.T))
    return out


def _oracle_grads(cfg, sd, x, dz, dtype, masks=None):
    import oracle.vqvae_cpu as ov
    m = ov.OracleVQVAE(cfg, sd)
    names = [n for n in m.params if n.startswith("encoder.")]
    with torch.no_grad():
        for n in names:
            m.params[n] = m.params[n].detach().to(dtype).requires_grad_(True)
    F0 = ov.F
    if masks is not None:
        ov.F = _FWithMasks(masks)
    try:
        z = m.encoder(x.to(dtype))
    finally:
        ov.F = F0
    g = torch.autograd.grad(z, [m.params[n] for n in names], grad_outputs=dz.to(dtype))
    return dict(zip(names, g)), z.detach()


@pytest.mark.parametrize("name", ["vcc20", "aishell3", "vcc20_multi"])
def test_encoder_backward_with_injected_dz_matches_float64(name):
    from oracle.vqvae_cpu import seeded_batch, seeded_state_dict
    from tests.helpers import cfg_of, make_trainer
    cfg = cfg_of(name, compute_dtype="fp32")
    wseed = 11
    B, T = 4, 128
    sd = seeded_state_dict(cfg, wseed)
    x, y = seeded_batch(cfg, B, T, 5)
    tr = make_trainer(cfg, wseed)
    eng = tr.engine
    torch.manual_seed(0)
    np.random.seed(0)
    w = eng.forward_train(x.cuda().contiguous(), y.cuda())
    Z, Tz = eng.dims["Z"], w.Tz
    g = torch.Generator().manual_seed(99)
    dz = torch.randn(B, Z, Tz, generator=g) / (B * Tz)          # dL/dz of a frame-mean loss, (B, Z, T_z)
    dz_ntc = dz.permute(0, 2, 1).reshape(B * Tz, Z).contiguous()
    eng.encoder_bwd(w, dz=dz_ntc.cuda())
    torch.cuda.synchronize()
    # LeakyReLU's derivative jumps at 0: a frame whose pre-activation is within
    # fp32 rounding of 0 may take either slope (and the two fp32 forwards may
    # disagree), so the float64 reference runs with the HIP forward's own sign
    # pattern -- the check is then exactly the Jacobian-vector product
    masks = hip_lrelu_masks(w)
    ref64, z64 = _oracle_grads(cfg, sd, x, dz, torch.float64, masks)
    ref32, _ = _oracle_grads(cfg, sd, x, dz, torch.float32, masks)
    # the forward the gradients flow through is the same one
    z_hip = w.z.view(B, Tz, Z).permute(0, 2, 1).double().cpu()
    assert float((z_hip - z64).abs().max() / z64.abs().max()) < 1e-5
    params = dict(tr.model.named_parameters())
    worst, worst_cpu, bad = 0.0, 0.0, []
    for n, r in ref64.items():
        got = eng.g(params[n]).double().cpu().view_as(r)
        scale = float(r.abs().max())
        if scale == 0.0:
            assert float(got.abs().max()) == 0.0, n
            continue
        err = float((got - r).abs().max()) / scale
        err_cpu = float((ref32[n].double() - r).abs().max()) / scale
        worst, worst_cpu = max(worst, err), max(worst_cpu, err_cpu)
        if err > BAR:
            bad.append((n, err, err_cpu))
    print(f"{name}: {len(ref64)} encoder tensors, worst HIP error {worst:.2e} (oracle fp32 CPU {worst_cpu:.2e})")
    assert not bad, bad
