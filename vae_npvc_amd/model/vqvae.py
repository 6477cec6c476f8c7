"""Drop-in `Model` for `model_type: vae_npvc_amd.model.vqvae` (the reference's
plugin seam, vae_npvc/trainer/basic.py:13,24-26): same constructor
`Model(arch_dict)`, same methods (forward / encode / decode / infer /
remove_weight_norm / load_state_dict, vqvae.py:11-119), same module tree and
state_dict keys (210 for the vcc20 config), so reference checkpoints load
unchanged.  The computation is the MI355X engine (vae_npvc_amd/engine/step.py);
there is no CPU implementation — calling the model on CPU tensors raises.

Extra config key (not in the reference YAMLs): `compute_dtype: fp32|bf16`
(default fp32 = the reference's arithmetic; bf16 runs the conv GEMMs on bf16
MFMA with fp32 accumulation, GroupNorm statistics, VQ and optimizer in fp32).
"""
import math

import torch
import torch.nn as nn

from ..engine.step import EngineOptions, VQVAEEngine
from .layers import Conditions, ResidualBlock, ResSkipBlock, WNConv1d
from .resample import ResampleConv1d
from .layers_vq import EMAVectorQuantizer, Jitter, VectorQuantizer


class Encoder(nn.Module):
    """vqvae.py:122-217: per resolution stage a conv (kernel_size, or the
    strided down-sampler of kernel 2s when the stage's downsample_scale s > 1,
    :146-157), `stacks` residual blocks with dilation 2**j (`dilation: true`)
    and `stack_layers` convs each, a LeakyReLU; then the 1x1 conv to
    z_channels.  Same nn.Sequential indices as the reference, so the
    state_dict keys match."""

    def __init__(self, in_channels=(513, 1024, 512, 256), out_channels=(1024, 512, 256, 128),
                 downsample_scales=(1, 1, 1, 1), kernel_size=3, z_channels=128, dilation=True, stack_kernel_size=3,
                 stack_layers=2, stacks=(3, 3, 3, 3), use_weight_norm=True, use_causal_conv=False):
        super().__init__()
        if use_causal_conv:
            raise NotImplementedError("Not supported yet.")  # vqvae.py:139
        wn = bool(use_weight_norm)  # false: plain convs with `weight` parameters (vqvae.py:179-180)
        layers, self.stage_index = [], []
        for cin, cout, ds, nst in zip(in_channels, out_channels, downsample_scales, stacks):
            self.stage_index.append(len(layers))
            if ds == 1:
                if (kernel_size - 1) % 2:
                    raise NotImplementedError("encoder: even kernel_size changes the frame count")
                layers.append(WNConv1d(cin, cout, kernel_size, weight_norm=wn))
            else:
                layers.append(ResampleConv1d(cin, cout, ds, weight_norm=wn))
            for j in range(nst):
                layers.append(ResidualBlock(cout, stack_kernel_size, stack_layers, 2 ** j if dilation else 1,
                                            weight_norm=wn))
            layers.append(nn.LeakyReLU(negative_slope=0.2))
        layers.append(WNConv1d(out_channels[-1], z_channels, 1, weight_norm=wn))
        self.encode = nn.Sequential(*layers)
        self.in_ch, self.z_ch = in_channels[0], z_channels


class Decoder(nn.Module):
    """vqvae.py:220-343: per stage a ConvTranspose1d (kernel_size, padding
    (k-1)//2; or the strided up-sampler of kernel 2s when upsample_scale
    s > 1, :245-265) and `stacks` ResSkip blocks with dilation 2**j; the skip
    outputs of all blocks are summed, scaled by sqrt(1/len(layers)) and sent
    through ReLU, 1x1, ReLU, 1x1 (:281-286, 308-318)."""

    def __init__(self, in_channels=(128, 256, 512, 1024), out_channels=(256, 512, 1024, 513),
                 upsample_scales=(1, 1, 1, 1), cond_channels=128, skip_channels=80, final_channels=80, kernel_size=5,
                 dilation=True, stack_kernel_size=3, stacks=(3, 3, 3, 3), use_weight_norm=True,
                 use_causal_conv=False):
        super().__init__()
        if use_causal_conv:
            raise NotImplementedError("Not supported yet.")  # vqvae.py:238
        wn = bool(use_weight_norm)  # false: plain convs with `weight` parameters (vqvae.py:290-293)
        layers, self.stage_index = [], []
        for cin, cout, us, nst in zip(in_channels, out_channels, upsample_scales, stacks):
            self.stage_index.append(len(layers))
            if us == 1:
                if (kernel_size - 1) % 2:
                    raise NotImplementedError("decoder: even kernel_size changes the frame count")
                layers.append(WNConv1d(cin, cout, kernel_size, transposed=True, weight_norm=wn))
            else:
                layers.append(ResampleConv1d(cin, cout, us, transposed=True, weight_norm=wn))
            for j in range(nst):
                layers.append(ResSkipBlock(cout, cond_channels, skip_channels, stack_kernel_size,
                                           2 ** j if dilation else 1, weight_norm=wn))
        self.layers = nn.ModuleList(layers)
        self.final_layer = nn.Sequential(nn.ReLU(), WNConv1d(skip_channels, skip_channels, 1, weight_norm=wn),
                                         nn.ReLU(), WNConv1d(skip_channels, final_channels, 1, weight_norm=wn))
        self.skip_ch, self.final_ch, self.cond_ch = skip_channels, final_channels, cond_channels


class _StepFunction(torch.autograd.Function):
    """Autograd bridge: the engine's fused forward saves every activation and
    its backward fills the flat gradient buffer; grads are returned per
    parameter so a stock torch optimizer (the reference Trainer) works too."""

    @staticmethod
    def forward(ctx, engine, x, y, *params):
        w = engine.forward_train(x, y)
        ctx.engine, ctx.w = engine, w
        total, vq = engine.total_loss(w)
        stats = w.stats.clone()
        ctx.mark_non_differentiable(vq, stats)
        return total.view(()), vq.view(()), stats

    @staticmethod
    def backward(ctx, g_total, g_vq, g_stats):
        eng, w = ctx.engine, ctx.w
        if g_total is None:
            return (None, None, None) + tuple(None for _ in eng.params)
        # The engine's backward assumes dL/dloss = 1; scale the flat gradient otherwise.
        eng.backward(w)
        grads = [eng.g(p).clone() for p in eng.params]
        if not torch.equal(g_total, torch.ones_like(g_total)):
            grads = [g * g_total for g in grads]
        return (None, None, None) + tuple(grads)


class Model(nn.Module):
    def __init__(self, arch):
        super().__init__()
        self.encoder = Encoder(**arch["encoder"])
        self.decoder = Decoder(**arch["decoder"])
        self.use_ema = arch.get("use_ema", False)
        # the reference's quantizers take any z_dim (layers_vq.py:166-173); the
        # fused VQ kernels (vqx_vq_forward) keep a frame's z_dim values in
        # registers and are built for 64, 128 and 256; the encoder's output
        # channels must equal z_dim, as the reference's quantizer needs
        z_dim, z_ch = arch.get("z_dim", 128), self.encoder.z_ch
        if z_dim not in (64, 128, 256) or z_ch != z_dim:
            raise NotImplementedError(f"z_dim {z_dim} / encoder output {z_ch}: the HIP quantizer is built for "
                                      "z_dim 64, 128 or 256 with the encoder's output channels equal to it")
        if self.use_ema:
            self.quantizer = EMAVectorQuantizer(arch.get("z_num", 512), arch.get("z_dim", 128), arch.get("mu", 0.9),
                                                reduction="frame_mean")
        else:  # straight-through codebook, L2-normalised by default (vqvae.py:26-32)
            self.quantizer = VectorQuantizer(arch.get("z_num", 512), arch.get("z_dim", 128),
                                             normalize=arch.get("embed_norm", True), reduction="frame_mean")
        self.embeds = Conditions(arch.get("y_num", 10), arch.get("y_dim", 128))
        self.jitter = Jitter(probability=arch.get("jitter_p", 0.0))
        self.beta = arch.get("beta", 0.01)
        self.compute_dtype = arch.get("compute_dtype", "fp32")
        # engine schedule options (engine/step.py EngineOptions; A/B runs only)
        self.engine_options = EngineOptions(**arch.get("engine", {}))
        self._engine = None

    # ------------------------------------------------------------ engine
    def engine(self, device=None):
        dev = device if device is not None else self.quantizer.embeddings.device
        if dev.type != "cuda":
            raise RuntimeError("vae_npvc_amd.Model runs only on the MI355X (HIP) path; move it with .cuda()")
        e = self._engine
        if e is None or e.device != dev or not e.params_intact():
            e = self._engine = VQVAEEngine(self, dev, self.compute_dtype, self.engine_options)
        return e

    # ------------------------------------------------------------ reference API
    def forward(self, input):
        """(x (B, mel, T), y (B, 1)) -> (xhat (B, mel, T), loss, loss dict) (vqvae.py:70-90)."""
        x, y_idx = input
        eng = self.engine(x.device)
        x = x.float().contiguous()
        if self.training:
            total, vq, stats = _StepFunction.apply(eng, x, y_idx, *eng.params)
            w = eng._ws[(x.shape[0], x.shape[2], True)]
            eng.vq_ema_update(w)  # update_emb runs inside the reference forward (layers_vq.py:295-296)
            stats = w.stats.clone()
            xhat = torch.empty_like(w.xhat_nct)
            from .. import ops
            ops.ntc_to_nct(w.xhat, xhat)
            detail = eng.loss_detail(w, stats.cpu())
            return xhat, total, detail
        w = eng.forward_eval(x, y_idx)
        d = eng.loss_detail(w, w.stats.cpu())
        detail = {k: d[k] for k in ("Total", "VQ loss", "X like")}
        if "entropy" in d and eng.plain:  # VectorQuantizer reports perplexity in eval too
            detail["entropy"] = d["entropy"]
        return w.xhat_nct.clone(), torch.tensor(d["Total"], device=x.device), detail

    def encode(self, input):
        x = input[0] if isinstance(input, (list, tuple)) else input
        return self.engine(x.device).encode(x.float().contiguous())

    def decode(self, input):
        z_idx, y_idx = input
        return self.engine(z_idx.device).decode(z_idx, y_idx)

    def infer(self, input):
        x, y_idx = input
        return self.decode((self.encode(x), y_idx))

    def remove_weight_norm(self):
        """vqvae.py:93-103: bake w = g*v/||v|| into a plain `weight` on every
        conv that has weight norm (stride-1 and resampling convs alike); the
        engine is rebuilt over the new parameters on its next use."""
        for m in self.modules():
            if isinstance(m, (WNConv1d, ResampleConv1d)) and m.has_weight_norm:
                m.remove_weight_norm()
        self._engine = None

    def load_state_dict(self, state_dict, strict=True):
        """vqvae.py:106-119: with the straight-through quantizer, a checkpoint
        whose codebook shape differs rebuilds the quantizer at that shape
        (same normalize / reduction) before loading; the engine re-flattens
        the parameters on its next use."""
        if not self.use_ema and "quantizer.embeddings" in state_dict:
            want = tuple(state_dict["quantizer.embeddings"].shape)
            have = tuple(self.quantizer.embeddings.shape)
            if want != have:
                print(f"Embedding size mismatch for model.quantizer: copying a param with shape {want} from "
                      f"checkpoint, resizing the param with shape {have} in current model.")
                dev = self.quantizer.embeddings.device
                self.quantizer = VectorQuantizer(want[0], want[1], normalize=self.quantizer.normalize,
                                                 reduction=self.quantizer.reduction).to(dev)
                self._engine = None
        out = super().load_state_dict(state_dict, strict=strict)
        if self._engine is not None:
            self._engine.invalidate_packed()
        return out


LOG_2PI = math.log(2.0 * math.pi)
