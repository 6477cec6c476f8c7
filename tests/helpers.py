"""Shared test helpers (configs, fixtures, seeded trainers)."""
import json
from pathlib import Path

import numpy as np
import torch
import yaml

ROOT = Path(__file__).resolve().parent.parent
GOLD = ROOT / "tests" / "golden"
CONF = ROOT / "vae_npvc_amd" / "conf"


# The general Encoder/Decoder topology of vqvae.py (fixtures
# tests/golden/step_vcc20_multi*): two resolution stages (the encoder
# down-samples by 2 in its second stage, the decoder up-samples by 2 in its
# first), dilation 2**j, stack_layers 2, the decoder's default kernel_size 5,
# mixed channel widths.
MULTI_ENC = {"in_channels": [80, 128], "out_channels": [128, 256], "downsample_scales": [1, 2], "kernel_size": 3,
             "z_channels": 128, "dilation": True, "stack_kernel_size": 3, "stack_layers": 2, "stacks": [2, 2],
             "use_weight_norm": True, "use_causal_conv": False}
MULTI_DEC = {"in_channels": [128, 256], "out_channels": [256, 128], "upsample_scales": [2, 1], "cond_channels": 64,
             "skip_channels": 64, "final_channels": 80, "kernel_size": 5, "dilation": True, "stack_kernel_size": 3,
             "stacks": [2, 2], "use_weight_norm": True, "use_causal_conv": False}
MULTI = {"vcc20_multi": ("vcc20", {"encoder": MULTI_ENC, "decoder": MULTI_DEC, "z_num": 128, "y_dim": 64,
                                   "jitter_p": 0.12}),
         "vcc20_multi_plain": ("vcc20", {"encoder": MULTI_ENC, "decoder": MULTI_DEC, "z_num": 128, "y_dim": 64,
                                         "use_ema": False})}


def _nown(base_cfg):
    """use_weight_norm: false in both halves (vqvae.py:179-180,290-293): plain Conv1d / ConvTranspose1d."""
    return {"encoder": dict(base_cfg["encoder"], use_weight_norm=False),
            "decoder": dict(base_cfg["decoder"], use_weight_norm=False)}


_VCC20 = yaml.safe_load(open(CONF / "vcc20.yaml"))
NOWN = {"vcc20_nown": ("vcc20", _nown(_VCC20)),
        "vcc20_multi_nown": ("vcc20_multi", dict(_nown({"encoder": MULTI_ENC, "decoder": MULTI_DEC})))}


def _zdim(base_cfg, z):
    """Codebook width z_dim = z (layers_vq.py:166-173): the encoder's output
    conv (z_channels) and the decoder's input (in_channels[0]) follow it."""
    return {"z_dim": z, "encoder": dict(base_cfg["encoder"], z_channels=z),
            "decoder": dict(base_cfg["decoder"], in_channels=[z])}


# z_dim 64 / 256 (the VQ kernels' other widths; fixtures tests/golden/step_vcc20_z*)
ZDIM = {"vcc20_z64": ("vcc20", _zdim(_VCC20, 64)), "vcc20_z256": ("vcc20", _zdim(_VCC20, 256)),
        "vcc20_z64_plain": ("vcc20_z64", {"use_ema": False}),
        "vcc20_z256_plain": ("vcc20_z256", {"use_ema": False})}


def cfg_of(name, **over):
    if name in NOWN or name in ZDIM:
        base, mo = NOWN[name] if name in NOWN else ZDIM[name]
        cfg = cfg_of(base)
        cfg.update(mo)
    elif name in MULTI:
        base, mo = MULTI[name]
        cfg = yaml.safe_load(open(CONF / f"{base}.yaml"))
        cfg.update(mo)
    else:
        cfg = yaml.safe_load(open(CONF / f"{name}.yaml"))
    cfg.update(over)
    return cfg


def load_fixture(prefix):
    meta = json.load(open(GOLD / f"{prefix}.json"))
    arr = dict(np.load(GOLD / f"{prefix}.npz", allow_pickle=False))
    return meta, arr


def relclose(a, b, rtol, atol=0.0):
    return abs(a - b) <= rtol * max(abs(b), 1e-12) + atol


def make_trainer(cfg, wseed):
    from oracle.vqvae_cpu import seeded_state_dict
    from vae_npvc_amd.trainer.basic import Trainer
    torch.manual_seed(0)
    tr = Trainer(cfg)
    tr.model.load_state_dict(seeded_state_dict(cfg, wseed))
    return tr


def oracle_step_grads(cfg, wseed, batch, tseed, nseed, bf16_autocast=False):
    """One oracle train step's (loss dict, per-parameter gradients).  With
    bf16_autocast the conv/matmul operands are rounded to bf16 with fp32
    accumulation (torch CPU autocast) and the quantizer stays fp32 -- the
    engine's bf16 policy restated in stock torch, i.e. the error a bf16 step
    has inherently (tools/bf16_autocast_ref.py)."""
    from oracle.vqvae_cpu import OracleTrainer, seeded_state_dict
    orc = OracleTrainer(dict(cfg, compute_dtype="fp32"), seeded_state_dict(cfg, wseed))
    if bf16_autocast:
        q0 = orc.model.quantize

        def q_fp32(z, _q=q0):
            with torch.autocast("cpu", enabled=False):
                return _q(z.float())
        orc.model.quantize = q_fp32
    torch.manual_seed(tseed)
    np.random.seed(nseed)
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16_autocast):
        _, det = orc.train_step(batch, keep_grads=True)
    return det, {k: v.detach().double() for k, v in orc.grads.items()}


def grad_errors(grads, ref):
    """Sorted per-parameter relative L2 errors [(err, name)] of grads vs ref."""
    out = []
    for n, r in ref.items():
        g = grads[n].detach().double().cpu()
        out.append((float((g - r).norm() / r.norm().clamp_min(1e-30)), n))
    return sorted(out)


NEAR_TIE = 1e-4  # a frame's top-2 relative distance gap below this is a near-tie (the training tests' bar)


def oracle_encode_gaps(orc, x):
    """(ids, top-2 relative gaps) of the oracle's Model.encode on x: the
    near-tie measure of the golden fixtures (make_golden.py Recorder), per frame
    in (utterance, time) order."""
    z = orc.encoder(x)
    zf = z.transpose(1, 2).contiguous().view(-1, z.shape[1])
    if orc.use_ema:
        E = orc.embeddings
    else:
        E = orc._plain_codebook(in_place=False)
        if orc.normalize:
            zf = zf / zf.norm(dim=1, keepdim=True)
    dist = orc.distances(zf, E)
    top2 = torch.topk(dist, 2, dim=1, largest=False).values
    gap = (top2[:, 1] - top2[:, 0]) / top2[:, 1].abs().clamp_min(1e-30)
    return torch.argmin(dist, dim=1).numpy(), gap.numpy()


def assert_ids_near_tie_exact(got, want, gap, what=""):
    """Every id that differs from the reference's sits at a reference near-tie."""
    got, want, gap = np.asarray(got).reshape(-1), np.asarray(want).reshape(-1), np.asarray(gap).reshape(-1)
    mism = got != want
    assert (gap[mism] < NEAR_TIE).all(), (what, int(mism.sum()), gap[mism][gap[mism] >= NEAR_TIE][:8])
    return int(mism.sum())
