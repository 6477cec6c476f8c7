"""Encoder backward at fp32 precision with an injected, well-conditioned dL/dz
(VERDICT r02 "weak #1").

In the training step the encoder's only gradient is beta * the commitment
term 2(z - z_q)/(B T) (layers_vq.py:301,315), a difference of nearly equal
vectors, so the step-level golden tests can only pin the encoder gradients to
~1e-3.  Here the SAME seeded dL/dz drives both the HIP encoder backward
(engine.encoder_bwd(dz=...): ten GroupNorm backwards, the fused DGRAD+WGRAD
launches, the split-K slabs and the weight-norm backward of every encoder
conv) and torch.autograd of the oracle encoder (vqvae.py:185-192,
layers.py:129-178) evaluated in float64.  Every encoder.* gradient must be
within 1e-5 of the float64 truth, elementwise, relative to the tensor's
largest entry; the oracle's own fp32 CPU gradients are reported beside it.
Recipes: vcc20 (config 2 widths), aishell3 (160 mel) and the general
two-stage topology (stride-2 resampling, dilation, stack_layers 2)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

BAR = 1e-5


def _oracle_grads(cfg, sd, x, dz, dtype):
    from oracle.vqvae_cpu import OracleVQVAE
    m = OracleVQVAE(cfg, sd)
    names = [n for n in m.params if n.startswith("encoder.")]
    with torch.no_grad():
        for n in names:
            m.params[n] = m.params[n].detach().to(dtype).requires_grad_(True)
    z = m.encoder(x.to(dtype))
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
    ref64, z64 = _oracle_grads(cfg, sd, x, dz, torch.float64)
    ref32, _ = _oracle_grads(cfg, sd, x, dz, torch.float32)
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
