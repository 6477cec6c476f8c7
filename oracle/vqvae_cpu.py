"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU fp32 restatement (plain torch-CPU ops) of the reference VQ-VAE training
step of Sinica-SLAM/vae_npvc, used as the parity checker for the HIP path
and as the CPU baseline timed by bench.py.  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product package
(vae_npvc_amd) never does.

Pinned against golden vectors produced by importing the reference itself in
the survey container (tests/golden/make_golden.py -> tests/golden/*.npz);
tests/test_oracle_golden.py checks this restatement against them.

Scope: the Encoder/Decoder of vqvae.py in
any topology the constructor accepts -- the single-stage recipes
(egs/vcc20/vae1, egs/aishell3/vc2) and the constructor defaults: several
resolution stages with strided down-/up-sampling convs, dilation 2**j,
stack_layers > 1, decoder kernel_size 5 -- EMAVectorQuantizer (use_ema: true) and the
straight-through VectorQuantizer (use_ema: false, embed_norm on/off), Jitter,
log_loss and Trainer.train_step (Adam, clip_grad_norm_, StepLR).  Every function cites the
reference file:line it restates (paths relative to the reference root).
"""
import math
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

LOG_2PI = math.log(2.0 * math.pi)  # vae_npvc/model/layers.py:8


# ----------------------------------------------------------------- structure
def encoder_plan(enc):
    """Encoder.__init__ (vqvae.py:123-183): per resolution stage a conv
    (kernel_size, or kernel 2s / stride s / padding s//2 + s%2 when the stage
    down-samples by s, :146-157), `stacks` Conv1d_Layernorm_LRelu_Residual
    blocks with dilation 2**j (`dilation: true`) and `stack_layers` convs each
    (layers.py:129-165), a LeakyReLU; then the 1x1 conv to z_channels.
    Returns (stages, final): stage = dict(idx, cin, cout, k, stride, pad,
    blocks=[dict(idx, dil)]); indices are positions in the nn.Sequential."""
    k0 = enc.get("kernel_size", 3)
    ks = enc.get("stack_kernel_size", 3)
    L = enc.get("stack_layers", 2)
    dil_on = enc.get("dilation", True)
    assert not enc.get("use_causal_conv", False) and (ks - 1) % 2 == 0
    stages, idx = [], 0
    for cin, cout, ds, nst in zip(enc["in_channels"], enc["out_channels"], enc.get("downsample_scales", [1] * 4),
                                  enc["stacks"]):
        if ds == 1:
            k, stride, pad = k0, 1, (k0 - 1) // 2
        else:
            k, stride, pad = 2 * ds, ds, ds // 2 + ds % 2
        st = dict(idx=idx, cin=cin, cout=cout, k=k, stride=stride, pad=pad, blocks=[], ks=ks, L=L)
        idx += 1
        for j in range(nst):
            st["blocks"].append(dict(idx=idx, dil=2 ** j if dil_on else 1))
            idx += 1
        idx += 1  # the stage's LeakyReLU
        stages.append(st)
    return stages, idx


def decoder_plan(dec):
    """Decoder.__init__ (vqvae.py:221-296): per stage a ConvTranspose1d
    (kernel_size, padding (k-1)//2; or kernel 2s / stride s / padding
    s//2 + s%2 / output_padding s%2 when the stage up-samples, :245-265) and
    `stacks` DeConv1d_Layernorm_GLU_ResSkip blocks with dilation 2**j
    (layers.py:181-215); positions are indices into the ModuleList."""
    k0 = dec.get("kernel_size", 5)
    ks = dec.get("stack_kernel_size", 3)
    dil_on = dec.get("dilation", True)
    assert not dec.get("use_causal_conv", False) and (ks - 1) % 2 == 0
    stages, idx = [], 0
    for cin, cout, us, nst in zip(dec["in_channels"], dec["out_channels"], dec.get("upsample_scales", [1] * 4),
                                  dec["stacks"]):
        if us == 1:
            k, stride, pad, opad = k0, 1, (k0 - 1) // 2, 0
        else:
            k, stride, pad, opad = 2 * us, us, us // 2 + us % 2, us % 2
        st = dict(idx=idx, cin=cin, cout=cout, k=k, stride=stride, pad=pad, opad=opad, blocks=[], ks=ks)
        idx += 1
        for j in range(nst):
            st["blocks"].append(dict(idx=idx, dil=2 ** j if dil_on else 1))
            idx += 1
        stages.append(st)
    return stages, idx


def layer_specs(cfg):
    """Ordered parameter spec [(name, shape)] of vae_npvc.model.vqvae.Model in
    registration order (== model.parameters() order; vqvae.py:15-40,
    layers.py:139-165,191-215; weight_norm registers weight_g/weight_v after
    bias), for any Encoder/Decoder topology of vqvae.py."""
    enc, dec = cfg["encoder"], cfg["decoder"]
    Z = enc.get("z_channels", 128)
    cond, skip, fin = dec["cond_channels"], dec["skip_channels"], dec["final_channels"]
    spec = []

    def conv(name, cin, cout, k, transposed=False, wn=True):
        v = (cin, cout, k) if transposed else (cout, cin, k)
        if not wn:  # plain nn.Conv1d / ConvTranspose1d registration: weight, bias (use_weight_norm: false)
            spec.append((name + ".weight", v))
            spec.append((name + ".bias", (cout,)))
            return
        spec.append((name + ".bias", (cout,)))
        g = (cin, 1, 1) if transposed else (cout, 1, 1)
        spec.append((name + ".weight_g", g))
        spec.append((name + ".weight_v", v))

    def gn(name, c):
        spec.append((name + ".weight", (c,)))
        spec.append((name + ".bias", (c,)))

    ewn, dwn = enc.get("use_weight_norm", True), dec.get("use_weight_norm", True)  # vqvae.py:179-180,290-293
    stages, fidx = encoder_plan(enc)
    for st in stages:
        C = st["cout"]
        conv(f"encoder.encode.{st['idx']}", st["cin"], C, st["k"], wn=ewn)
        for b in st["blocks"]:
            pre = f"encoder.encode.{b['idx']}"
            for l in range(st["L"]):
                conv(f"{pre}.stack.{3 * l + 1}", C, C, st["ks"], wn=ewn)
                gn(f"{pre}.stack.{3 * l + 2}", C)
            conv(f"{pre}.skip_layer", C, C, 1, wn=ewn)
    conv(f"encoder.encode.{fidx}", enc["out_channels"][-1], Z, 1, wn=ewn)
    for st in decoder_plan(dec)[0]:
        C = st["cout"]
        conv(f"decoder.layers.{st['idx']}", st["cin"], C, st["k"], transposed=True, wn=dwn)
        for b in st["blocks"]:
            pre = f"decoder.layers.{b['idx']}"
            conv(f"{pre}.conv_in", C, 2 * C, st["ks"], transposed=True, wn=dwn)
            gn(f"{pre}.norm_layer", 2 * C)
            conv(f"{pre}.conv_cond", cond, 2 * C, 1, wn=dwn)
            conv(f"{pre}.res_skip_layers", C, C + skip, 1, wn=dwn)
    conv("decoder.final_layer.1", skip, skip, 1, wn=dwn)
    conv("decoder.final_layer.3", skip, fin, 1, wn=dwn)
    if not cfg.get("use_ema", False):  # VectorQuantizer's codebook is a parameter (layers_vq.py:18)
        spec.append(("quantizer.embeddings", (cfg.get("z_num", 512), cfg.get("z_dim", 128))))
    spec.append(("embeds._embedding.weight", (cfg.get("y_num", 10), cfg.get("y_dim", 128))))
    return spec


def buffer_specs(cfg):
    K, D = cfg.get("z_num", 512), cfg.get("z_dim", 128)
    if not cfg.get("use_ema", False):
        return []
    return [("quantizer.emb_init", ()), ("quantizer.emb_sum", (K, D)), ("quantizer.emb_elem", (K,)),
            ("quantizer.embeddings", (K, D))]


def _is_gn(name):  # GroupNorm affine parameters: stack.{2,5,8,..} and norm_layer
    parts = name.split(".")
    return "norm_layer" in parts or ("stack" in parts and int(parts[parts.index("stack") + 1]) % 3 == 2)


def seeded_state_dict(cfg, seed):
    """Deterministic weights from a numpy PCG64 stream (platform independent),
    shaped like the reference default init: v ~ U(-1/sqrt(fan_in), +), g =
    ||v_o|| * U(0.8, 1.2), biases U(-b, b), GroupNorm affine near (1, 0),
    embedding N(0, 1).  Fresh EMA buffers (layers_vq.py:170-173)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sd = OrderedDict()
    for name, shape in layer_specs(cfg):
        if name.endswith(".weight_v"):
            fan_in = int(np.prod(shape[1:]))  # torch's fan_in for Conv1d and ConvTranspose1d weights
            b = 1.0 / math.sqrt(fan_in)
            v = rng.uniform(-b, b, size=shape).astype(np.float32)
            sd[name] = torch.from_numpy(v)
            g = sd[name[:-1] + "g"]
            norm = np.sqrt((v.astype(np.float64) ** 2).reshape(shape[0], -1).sum(1)).astype(np.float32)
            sd[name[:-1] + "g"] = torch.from_numpy((norm * g.numpy().reshape(-1)).reshape(g.shape).astype(np.float32))
        elif name.endswith(".weight_g"):
            sd[name] = torch.from_numpy(rng.uniform(0.8, 1.2, size=shape).astype(np.float32))
        elif name.endswith(".bias") and _is_gn(name):
            sd[name] = torch.from_numpy((0.1 * rng.standard_normal(shape)).astype(np.float32))
        elif name.endswith(".weight") and _is_gn(name):
            sd[name] = torch.from_numpy((1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32))
        elif name.endswith(".bias"):
            sd[name] = torch.from_numpy(rng.uniform(-0.05, 0.05, size=shape).astype(np.float32))
        elif name in ("embeds._embedding.weight", "quantizer.embeddings"):
            sd[name] = torch.from_numpy(rng.standard_normal(shape).astype(np.float32))
        elif name.endswith(".weight"):  # a conv without weight norm: U(-1/sqrt(fan_in), +)
            b = 1.0 / math.sqrt(int(np.prod(shape[1:])))
            sd[name] = torch.from_numpy(rng.uniform(-b, b, size=shape).astype(np.float32))
        else:
            raise KeyError(name)
    K, D = cfg.get("z_num", 512), cfg.get("z_dim", 128)
    if not cfg.get("use_ema", False):
        return sd
    sd["quantizer.emb_init"] = torch.tensor(False)
    sd["quantizer.emb_sum"] = torch.zeros(K, D)
    sd["quantizer.emb_elem"] = torch.ones(K)
    sd["quantizer.embeddings"] = torch.zeros(K, D)
    return sd


def seeded_batch(cfg, B, T, seed):
    """Synthetic CMVN-like mel batch x ~ N(0,1) (B, mel, T) f32 and speaker ids
    y (B, 1) int64 (the utt2mel_spk.py:42-74 contract)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    mel = cfg["encoder"]["in_channels"][0]
    x = rng.standard_normal((B, mel, T)).astype(np.float32)
    y = rng.integers(0, cfg.get("y_num", 10), size=(B, 1)).astype(np.int64)
    return torch.from_numpy(x), torch.from_numpy(y)


# ----------------------------------------------------------------- the model
class OracleVQVAE:
    """Functional restatement of vae_npvc.model.vqvae.Model with the EMA
    quantizer (use_ema: true) or the straight-through VectorQuantizer
    (use_ema: false).  Parameters are CPU fp32 leaf tensors keyed by the
    reference state_dict names."""

    def __init__(self, cfg, state_dict):
        self.cfg = cfg
        self.params = OrderedDict()
        for name, shape in layer_specs(cfg):
            t = state_dict[name].detach().clone().float().contiguous()
            assert tuple(t.shape) == tuple(shape), (name, t.shape, shape)
            self.params[name] = t.requires_grad_(True)
        self.use_ema = cfg.get("use_ema", False)
        self.normalize = cfg.get("embed_norm", True)  # vqvae.py:30
        if self.use_ema:
            self.emb_init = bool(state_dict["quantizer.emb_init"])
            self.emb_sum = state_dict["quantizer.emb_sum"].clone().float()
            self.emb_elem = state_dict["quantizer.emb_elem"].clone().float()
            self.embeddings = state_dict["quantizer.embeddings"].clone().float()
        self.mu = cfg.get("mu", 0.9)
        self.beta = cfg.get("beta", 0.01)
        self.jitter_p = cfg.get("jitter_p", 0.0)
        self.K, self.D = cfg.get("z_num", 512), cfg.get("z_dim", 128)
        self.threshold = 1.0
        self.training = True
        self.last = {}

    def state_dict(self):
        sd = OrderedDict((k, v.detach().clone()) for k, v in self.params.items())
        if not self.use_ema:
            return sd
        sd["quantizer.emb_init"] = torch.tensor(self.emb_init)
        sd["quantizer.emb_sum"] = self.emb_sum.clone()
        sd["quantizer.emb_elem"] = self.emb_elem.clone()
        sd["quantizer.embeddings"] = self.embeddings.clone()
        return sd

    # nn.utils.weight_norm pre-hook, torch._weight_norm(v, g, dim=0)
    def _w(self, name):
        if name + ".weight" in self.params:  # use_weight_norm: false
            return self.params[name + ".weight"]
        return torch._weight_norm(self.params[name + ".weight_v"], self.params[name + ".weight_g"], 0)

    def _conv(self, x, name, pad, transposed=False, stride=1, dilation=1, output_padding=0):
        if transposed:
            return F.conv_transpose1d(x, self._w(name), self.params[name + ".bias"], stride=stride, padding=pad,
                                      output_padding=output_padding, dilation=dilation)
        return F.conv1d(x, self._w(name), self.params[name + ".bias"], stride=stride, padding=pad,
                        dilation=dilation)

    # vqvae.py:185-192 with the Sequential of :144-176; block layers.py:168-178
    def encoder(self, x):
        p = self.params
        stages, fidx = encoder_plan(self.cfg["encoder"])
        h = x
        for si, st in enumerate(stages):
            if si > 0:
                h = F.leaky_relu(h, 0.2)  # the previous stage's trailing LeakyReLU (vqvae.py:171)
            h = self._conv(h, f"encoder.encode.{st['idx']}", st["pad"], stride=st["stride"])
            ks = st["ks"]
            for b in st["blocks"]:
                pre = f"encoder.encode.{b['idx']}"
                a = h
                for l in range(st["L"]):  # layers.py:151-161
                    dil = b["dil"] if l == 0 else 1
                    a = F.leaky_relu(a, 0.2)
                    a = self._conv(a, f"{pre}.stack.{3 * l + 1}", (ks - 1) // 2 * dil, dilation=dil)
                    a = F.group_norm(a, 1, p[f"{pre}.stack.{3 * l + 2}.weight"], p[f"{pre}.stack.{3 * l + 2}.bias"],
                                     1e-5)
                h = a + self._conv(h, pre + ".skip_layer", 0)
        h = F.leaky_relu(h, 0.2)
        return self._conv(h, f"encoder.encode.{fidx}", 0)

    # vqvae.py:298-318; block layers.py:218-249
    def decoder(self, zq, c):
        p = self.params
        stages, n_layers = decoder_plan(self.cfg["decoder"])
        c = c[:, :, :1]
        x_out = 0.0
        x = zq
        for st in stages:
            x = self._conv(x, f"decoder.layers.{st['idx']}", st["pad"], transposed=True, stride=st["stride"],
                           output_padding=st["opad"])
            T = x.size(2)
            Cd = x.size(1)
            ks = st["ks"]
            for b in st["blocks"]:
                pre = f"decoder.layers.{b['idx']}"
                dil = b["dil"]
                xr = self._conv(x, pre + ".conv_in", (ks - 1) // 2 * dil, transposed=True, dilation=dil)
                xc = self._conv(c.repeat(1, 1, T), pre + ".conv_cond", 0)
                h = F.group_norm(xr + xc, 2, p[pre + ".norm_layer.weight"], p[pre + ".norm_layer.bias"], 1e-5)
                g = torch.tanh(h[:, :Cd]) * torch.sigmoid(h[:, Cd:])
                r = self._conv(g, pre + ".res_skip_layers", 0)
                x = r[:, :Cd, :] + x
                x_out += r[:, Cd:, :]
        x = x_out * math.sqrt(1.0 / n_layers)
        x = F.relu(x)
        x = self._conv(x, "decoder.final_layer.1", 0)
        x = F.relu(x)
        return self._conv(x, "decoder.final_layer.3", 0)

    # ---- EMAVectorQuantizer (layers_vq.py:166-334)
    def _tile(self, z):  # layers_vq.py:183-190
        n, d = z.shape
        if n < self.K:
            rep = (self.K + n - 1) // n
            std = 0.01 / np.sqrt(d)
            z = z.repeat(rep, 1)
            z = z + torch.randn_like(z) * std
        return z

    # Data-parallel hooks (tests/test_ddp_gloo.py): identity in one process.
    # reduce_sum all-reduces the EMA statistics; pick_rows draws the
    # dead-code / init rows z[randperm(N)[:K]] from the GLOBAL batch.
    def reduce_sum(self, t):
        return t

    def pick_rows(self, z):  # _tile (noise drawn first), then randperm (layers_vq.py:197,212-213)
        zt = self._tile(z)
        return zt[torch.randperm(zt.shape[0])][: self.K]

    def init_emb(self, z):  # layers_vq.py:192-201
        self.emb_init = not self.emb_init
        self.embeddings = self.pick_rows(z)
        self.emb_sum = self.embeddings.clone()
        self.emb_elem = torch.ones(self.K)

    def update_emb(self, z, idx):  # layers_vq.py:203-233
        mu, K, D = self.mu, self.K, self.D
        with torch.no_grad():
            onehot = torch.zeros(K, z.shape[0])
            onehot.scatter_(0, idx.view(1, z.shape[0]), 1)
            s = self.reduce_sum(torch.matmul(onehot, z))
            n = self.reduce_sum(onehot.sum(dim=-1))
            rand = self.pick_rows(z)
            old = self.embeddings.clone()
            self.emb_sum = mu * self.emb_sum + (1.0 - mu) * s
            self.emb_elem = mu * self.emb_elem + (1.0 - mu) * n
            usage = (self.emb_elem.view(K, 1) >= self.threshold).float()
            self.embeddings = usage * (self.emb_sum.view(K, D) / self.emb_elem.view(K, 1)) + (1 - usage) * rand
            kp = n / torch.sum(n)
            entropy = torch.exp(-torch.sum(kp * torch.log(kp + 1e-8)))
            used_curr = (n >= self.threshold).sum()
            usage = torch.sum(usage)
            dk = torch.norm(self.embeddings - old) / np.sqrt(np.prod(old.shape))
        return {"entropy": entropy.item(), "used_curr": used_curr.item(), "usage": usage.item(), "diff_emb": dk.item()}

    def distances(self, zf, E):  # layers_vq.py:285-289
        return (torch.sum(zf.pow(2), dim=1, keepdim=True) + torch.sum(E.pow(2), dim=1) - 2 * torch.matmul(zf, E.t()))

    def quantize(self, z):  # layers_vq.py:268-323 (reduction 'frame_mean')
        B, D, T = z.shape
        zf = z.transpose(1, 2).contiguous().view(-1, D)
        if not self.emb_init and self.training:
            self.init_emb(zf)
        with torch.no_grad():
            dist = self.distances(zf, self.embeddings)
            idx = torch.argmin(dist, dim=1)
            zq = self.embeddings.index_select(dim=0, index=idx)
        self.last["idx"] = idx.detach().clone()
        self.last["dist"] = dist
        detail = self.update_emb(zf, idx) if self.training else {}
        enc_loss = F.mse_loss(zq.detach(), zf, reduction="none").sum() / (B * T)
        zq = zq.view(B, T, D).transpose(1, 2).contiguous()
        return zq, 0.0, enc_loss, detail

    # ---- VectorQuantizer (layers_vq.py:9-163), reduction 'frame_mean', target_norm 1.0
    def _plain_codebook(self, in_place):
        E = self.params["quantizer.embeddings"]
        if not self.normalize:
            return E
        if in_place:  # embed_norm() (layers_vq.py:28-33), called by every forward
            with torch.no_grad():
                E.mul_(1.0 / E.norm(dim=1, keepdim=True))
        return 1.0 * E / E.norm(dim=1, keepdim=True)

    def quantize_plain(self, z):  # layers_vq.py:79-150
        B, D, T = z.shape
        zf = z.transpose(1, 2).contiguous().view(-1, D)
        z_norm = 1.0 * zf / zf.norm(dim=1, keepdim=True) if self.normalize else zf
        emb = self._plain_codebook(in_place=True)
        dist = self.distances(z_norm, emb)
        idx = torch.argmin(dist, dim=1)
        z_vq = emb.index_select(dim=0, index=idx)
        self.last["idx"] = idx.detach().clone()
        counts = torch.bincount(idx, minlength=self.K).float()
        avg_probs = counts / idx.numel()
        perplexity = torch.exp(-torch.sum(avg_probs * torch.log(avg_probs + 1e-10)))
        z_qut_loss = F.mse_loss(z_vq, z_norm.detach(), reduction="none")
        z_enc_loss = F.mse_loss(z_vq.detach(), z_norm, reduction="none")
        if self.normalize:
            z_enc_loss = z_enc_loss + F.mse_loss(z_norm, zf, reduction="none")
        z_qut_loss = z_qut_loss.sum() / (B * T)
        z_enc_loss = z_enc_loss.sum() / (B * T)
        z_vq = z_norm + (z_vq - z_norm).detach()
        z_vq = z_vq.view(B, T, D).transpose(1, 2).contiguous()
        return z_vq, z_qut_loss, z_enc_loss, {"entropy": perplexity.item()}

    def encode(self, x):  # vqvae.py:45-52 / layers_vq.py:236-252 (EMA), 36-58 (plain)
        z = self.encoder(x)
        B, D, T = z.shape
        zf = z.transpose(1, 2).contiguous().view(-1, D)
        if self.use_ema:
            return torch.argmin(self.distances(zf, self.embeddings), dim=1).view(B, T)
        if self.normalize:
            zf = 1.0 * zf / zf.norm(dim=1, keepdim=True)
        return torch.argmin(self.distances(zf, self._plain_codebook(in_place=False)), dim=1).view(B, T)

    def decode(self, z_idx, y_idx):  # vqvae.py:55-60 / layers_vq.py:255-265 (EMA), 61-76 (plain)
        y = F.embedding(y_idx, self.params["embeds._embedding.weight"]).transpose(1, 2).contiguous()
        B, T = z_idx.shape
        E = self.embeddings if self.use_ema else self._plain_codebook(in_place=False)
        zq = E.index_select(0, z_idx.flatten()).view(B, T, -1).transpose(1, 2).contiguous()
        return self.decoder(zq, y)

    def jitter(self, zq):  # layers_vq.py:353-379 (replaces with probability 1-p: the reference's quirk)
        p = self.jitter_p
        if p == 0.0 or not self.training:
            return zq
        orig = zq.detach().clone()
        L = orig.size(2)
        for i in range(L):
            replace = [True, False][np.random.choice([1, 0], p=[p, 1 - p])]
            if replace:
                if i == 0:
                    nb = i + 1
                elif i == L - 1:
                    nb = i - 1
                else:
                    nb = i + np.random.choice([-1, 1], p=[0.5, 0.5])
                zq[:, :, i] = orig[:, :, nb]
        return zq

    def forward(self, x, y_idx):  # vqvae.py:70-90
        y = F.embedding(y_idx, self.params["embeds._embedding.weight"]).transpose(1, 2).contiguous()
        z = self.encoder(x)
        self.last["z"] = z
        zq, zq_loss, enc_loss, detail = self.quantize(z) if self.use_ema else self.quantize_plain(z)
        zq = self.jitter(zq)
        xhat = self.decoder(zq, y)
        B, D, T = x.shape
        x_loss = (0.5 * (LOG_2PI + (xhat - x).pow(2))).sum() / (B * T)  # layers.py:283-296
        loss = x_loss + zq_loss + self.beta * enc_loss
        losses = {"Total": loss.item(), "VQ loss": enc_loss.item(), "X like": x_loss.item()}
        losses.update(detail)
        return xhat, loss, losses


class ORAdam(torch.optim.Optimizer):
    """RAdam.step (trainer/radam.py:15-78) in the same fp32 op order, on the
    current torch signatures: v = v*b2 + (1-b2)*g*g, m = m*b1 + (1-b1)*g,
    N_sma = N_max - 2 t b2^t / (1 - b2^t); N_sma >= 5: p += -(ss*lr) * m /
    (sqrt(v) + eps) with the rectified step size ss (python doubles, :53-57),
    else p += -(lr/(1 - b1^t)) * m (:58-59, 68-71).  weight_decay 0 only
    (trainer/basic.py:31-34)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0):
        assert weight_decay == 0
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self):
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                grad = p.grad.float()
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                m, v = st["exp_avg"], st["exp_avg_sq"]
                v.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
                m.mul_(beta1).add_(grad, alpha=1 - beta1)
                st["step"] += 1
                t = st["step"]
                beta2_t = beta2 ** t
                n_max = 2 / (1 - beta2) - 1
                n_sma = n_max - 2 * t * beta2_t / (1 - beta2_t)
                if n_sma >= 5:
                    ss = math.sqrt((1 - beta2_t) * (n_sma - 4) / (n_max - 4) * (n_sma - 2) / n_sma * n_max /
                                   (n_max - 2)) / (1 - beta1 ** t)
                    p.addcdiv_(m, v.sqrt().add_(group["eps"]), value=-ss * group["lr"])
                else:
                    ss = 1.0 / (1 - beta1 ** t)
                    p.add_(m, alpha=-ss * group["lr"])


class OracleTrainer:
    """Trainer.train_step (trainer/basic.py:55-79) on CPU: zero_grad, forward,
    backward, clip_grad_norm_, Adam or RAdam (betas=(0.5, 0.999), wd 0,
    trainer/basic.py:30-39), StepLR."""

    def __init__(self, cfg, state_dict):
        self.model = OracleVQVAE(cfg, state_dict)
        params = list(self.model.params.values())
        self.max_grad_norm = cfg.get("max_grad_norm", 5)
        if str(cfg.get("optim_type", "Adam")).upper() == "RADAM":
            self.optimizer = ORAdam(params, lr=cfg.get("learning_rate", 1e-3), betas=(0.5, 0.999), weight_decay=0.0)
        else:
            self.optimizer = torch.optim.Adam(params, lr=cfg.get("learning_rate", 1e-3), betas=(0.5, 0.999),
                                              weight_decay=0.0)
        self.scheduler = None
        if cfg.get("lr_scheduler", None) is not None:
            lp = cfg.get("lr_param", {"step_size": 100000, "gamma": 0.5, "last_epoch": -1})
            self.scheduler = torch.optim.lr_scheduler.StepLR(optimizer=self.optimizer, **lp)
        self.iteration = 0
        self.grads = None
        self.grad_hook = None

    def train_step(self, batch, keep_grads=False):
        for p in self.model.params.values():
            p.grad = None
        x, y = batch
        xhat, loss, detail = self.model.forward(x, y)
        loss.backward()
        if self.grad_hook is not None:  # data parallel: gradient all-reduce (mean)
            self.grad_hook(list(self.model.params.values()))
        if keep_grads:
            self.grads = OrderedDict((k, v.grad.detach().clone()) for k, v in self.model.params.items())
        if self.max_grad_norm > 0:
            torch.nn.utils.clip_grad_norm_(list(self.model.params.values()), self.max_grad_norm)
        self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()
        self.iteration += 1
        self.last_xhat = xhat.detach()
        return self.iteration, detail
