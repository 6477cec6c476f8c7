"""Generate the golden fixtures of tests/golden/ by running the REFERENCE
implementation (Sinica-SLAM/vae_npvc, read-only at /root/reference) on CPU.

Run in the survey/build container only (the reference never travels):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it records (all inputs are regenerated from seeds, so only outputs are
stored):
  * structure.json        reference Model state_dict keys/shapes/order per config
  * step_<cfg>.npz/.json  3 training steps of Model + a restatement of
                          Trainer.train_step (trainer/basic.py:55-79 without
                          .cuda(), which is hard-coded there) from
                          oracle.seeded_state_dict / seeded_batch
  * vq_K<k>.npz/.json     EMAVectorQuantizer.forward (layers_vq.py:268-323) at
                          N = 16384 frames, K in {128, 512, 1024}
  * vq_tile.npz/.json     the N < K tiling path (layers_vq.py:183-190)
  * jitter.json           Jitter.forward neighbour map (layers_vq.py:353-379)
  * full_step.npz/.json   2 steps at the config-2 size B=64 x T=256
  * full_step_vcc20_b512  2 steps at B=512 x T=256 (--only-big): config 3's
                          global batch (8 ranks x 64 x 256), pinning the
                          single-process engine and the 8-rank data-parallel
                          engine at config 3's real partition (≈22 GB of
                          RAM for the reference's CPU autograd)
  * step_<cfg>_plain*     3 steps with the straight-through VectorQuantizer
                          (use_ema: false; embed_norm true / false; aishell3
                          with jitter_p 0.12), SURVEY §8f row 1
  * step_vcc20_radam      8 steps with optim_type RAdam (trainer/radam.py,
                          SURVEY §8f row 4); RAdam switches to the adaptive
                          update at step 6
  * step_vcc20_z*         3 steps at codebook width z_dim 64 / 256, EMA and
                          straight-through quantizers (--only-zdim)
  * encode_<cfg>          Model.encode ids + top-2 gaps and Model.decode of
                          them, eval mode, odd lengths (--only-encode), the
                          inference path of bin/extract_bnf.py (§8f row 3)
  * step_vcc20_multi*     3 steps of the general Encoder/Decoder topology
                          (two resolution stages with strided resampling
                          convs, dilation 2**j, stack_layers 2, decoder
                          kernel 5; EMA + jitter, and straight-through VQ),
                          SURVEY §8f row 4 (--only-multi)
Weights/inputs come from numpy PCG64 seeds (oracle/vqvae_cpu.py), so the GPU
box regenerates them bit-identically without receiving any weights.
"""
import json
import os
import sys
import warnings
from pathlib import Path

import numpy as np
import torch
import yaml

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
REF = Path(os.environ.get("VQX_REFERENCE", "/root/reference"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(REF))
warnings.filterwarnings("ignore")

from oracle.vqvae_cpu import buffer_specs, layer_specs, seeded_batch, seeded_state_dict  # noqa: E402

CFGS = {
    "vcc20": REF / "egs/vcc20/vae1/conf/train_pytorch_vqvae.yaml",
    "aishell3": REF / "egs/aishell3/vc2/conf/train_pytorch_vqvae.yaml",
}


VARIANTS = {  # derived configs: base recipe + overrides
    "vcc20_plain": ("vcc20", {"use_ema": False}),
    "vcc20_plain_nonorm": ("vcc20", {"use_ema": False, "embed_norm": False}),
    "aishell3_plain": ("aishell3", {"use_ema": False}),
}
RADAM = {"vcc20_radam": ("vcc20", {"optim_type": "RAdam"})}
from tests.helpers import MULTI, NOWN, ZDIM  # noqa: E402  (general topology; no weight norm; z_dim)
VARIANTS_ALL = dict(VARIANTS, **RADAM, **MULTI, **NOWN, **ZDIM)


def load_cfg(name):
    if name in VARIANTS_ALL:
        base, over = VARIANTS_ALL[name]
        cfg = load_cfg(base) if base in VARIANTS_ALL else yaml.safe_load(open(CFGS[base]))
        cfg.update(over)
        return cfg
    return yaml.safe_load(open(CFGS[name]))


def ref_model(cfg, sd):
    from vae_npvc.model.vqvae import Model
    m = Model(cfg)
    m.load_state_dict(sd)
    m.train()
    return m


class Recorder:
    """Wraps quantizer.update_emb to capture (z, idx, E_used) of each step."""

    def __init__(self, q):
        self.q = q
        self.orig = q.update_emb
        self.calls = []
        q.update_emb = self

    def __call__(self, z, z_idx):
        E = self.q.embeddings.detach().clone()
        z = z.detach()
        dist = (z.pow(2).sum(1, keepdim=True) + E.pow(2).sum(1)) - 2 * z @ E.t()
        top2 = torch.topk(dist, 2, dim=1, largest=False).values
        gap = (top2[:, 1] - top2[:, 0]) / top2[:, 1].abs().clamp_min(1e-30)
        self.calls.append(dict(idx=z_idx.detach().clone(), z=z.clone(), E=E, gap=gap))
        return self.orig(z, z_idx)


def ref_train_step(model, opt, sched, batch, max_grad_norm):
    """trainer/basic.py:55-79 on CPU."""
    model.zero_grad()
    out, loss, detail = model(list(batch))
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
    if max_grad_norm > 0:
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_grad_norm)
    opt.step()
    if sched is not None:
        sched.step()
    return out.detach(), detail, grads


def summarize(t, n=16):
    t = t.detach().double().reshape(-1)
    return dict(norm=float(t.norm()), sum=float(t.sum()), head=[float(v) for v in t[:n]])


def step_fixture(name, B, T, steps, wseed, bseed, tseed, nseed, out_prefix, keep_idx=True, compact=False):
    """compact (the B=512 fixture): xhat slice of the first 64 utterances only,
    top-2 gaps as float16 (the tests only ask whether a gap is < 1e-4)."""
    cfg = load_cfg(name)
    sd = seeded_state_dict(cfg, wseed)
    model = ref_model(cfg, sd)
    assert [k for k, _ in model.named_parameters()] == [k for k, _ in layer_specs(cfg)], "parameter order"
    ema = cfg.get("use_ema", False)
    rec = Recorder(model.quantizer) if ema else None
    if str(cfg.get("optim_type", "Adam")).upper() == "RADAM":  # trainer/basic.py:30-34
        from vae_npvc.trainer.radam import RAdam
        opt = RAdam(model.parameters(), lr=cfg.get("learning_rate", 1e-3), betas=(0.5, 0.999), weight_decay=0.0)
    else:
        opt = torch.optim.Adam(model.parameters(), lr=cfg.get("learning_rate", 1e-3), betas=(0.5, 0.999),
                               weight_decay=0.0)
    sched = torch.optim.lr_scheduler.StepLR(optimizer=opt, **cfg["lr_param"]) if cfg.get("lr_scheduler") else None
    torch.manual_seed(tseed)
    np.random.seed(nseed)
    meta = dict(config=name, B=B, T=T, steps=steps, wseed=wseed, bseed=bseed, tseed=tseed, nseed=nseed,
                torch=torch.__version__, numpy=np.__version__, detail=[], grads={}, params_after={}, xhat={})
    arrays = {}
    for s in range(steps):
        batch = seeded_batch(cfg, B, T, bseed + s)
        xhat, detail, grads = ref_train_step(model, opt, sched, batch, cfg.get("max_grad_norm", 5))
        meta["detail"].append({k: float(v) for k, v in detail.items()})
        meta["xhat"][str(s)] = summarize(xhat)
        if s == 0:
            meta["grads"] = {k: summarize(g) for k, g in grads.items()}
            arrays["xhat0_slice"] = xhat[:64 if compact else B, :, :16].numpy().astype(np.float32)
        q = model.quantizer
        meta[f"embeddings{s}"] = summarize(q.embeddings)
        if not ema:
            continue
        c = rec.calls[-1]
        if keep_idx:
            arrays[f"idx{s}"] = c["idx"].numpy().astype(np.int16)
            arrays[f"gap{s}"] = c["gap"].numpy().astype(np.float16 if compact else np.float32)
        arrays[f"emb_elem{s}"] = q.emb_elem.detach().numpy().astype(np.float32)
        meta[f"emb_sum{s}"] = summarize(q.emb_sum)
    meta["params_after"] = {k: summarize(p, 8) for k, p in model.named_parameters()}
    np.savez_compressed(HERE / f"{out_prefix}.npz", **arrays)
    json.dump(meta, open(HERE / f"{out_prefix}.json", "w"), indent=1)
    print(f"[golden] {out_prefix}: {[round(d['Total'], 5) for d in meta['detail']]}")


def vq_fixture(K, N_B, N_T, seed, out_prefix):
    from vae_npvc.model.layers_vq import EMAVectorQuantizer
    D = 128
    rng = np.random.Generator(np.random.PCG64(seed))
    z = torch.from_numpy(rng.standard_normal((N_B, D, N_T)).astype(np.float32))
    E = torch.from_numpy(rng.standard_normal((K, D)).astype(np.float32))
    emb_sum = torch.from_numpy((1.5 * rng.standard_normal((K, D))).astype(np.float32))
    emb_elem = torch.from_numpy(rng.uniform(0.5, 3.0, size=(K,)).astype(np.float32))
    q = EMAVectorQuantizer(K, D, 0.9, reduction="frame_mean")
    q.emb_init = torch.tensor(True)
    q.embeddings = E.clone()
    q.emb_sum = emb_sum.clone()
    q.emb_elem = emb_elem.clone()
    q.train()
    rec = Recorder(q)
    idx_eval = q.encode(z)
    torch.manual_seed(seed + 1)
    zq, _, enc_loss, detail = q(z)
    c = rec.calls[-1]
    arrays = dict(idx=c["idx"].numpy().astype(np.int16), gap=c["gap"].numpy().astype(np.float32),
                  idx_eval=idx_eval.reshape(-1).numpy().astype(np.int16),
                  emb_elem=q.emb_elem.numpy().astype(np.float32),
                  emb_row_norm=q.embeddings.norm(dim=1).numpy().astype(np.float32),
                  emb_sum_row_norm=q.emb_sum.norm(dim=1).numpy().astype(np.float32),
                  emb_head=q.embeddings[:4].numpy().astype(np.float32))
    meta = dict(K=K, D=D, B=N_B, T=N_T, seed=seed, torch_seed=seed + 1, enc_loss=float(enc_loss),
                detail={k: float(v) for k, v in detail.items()}, zq=summarize(zq),
                embeddings=summarize(q.embeddings), emb_sum=summarize(q.emb_sum),
                min_gap=float(c["gap"].min()), n_gap_lt_1e5=int((c["gap"] < 1e-5).sum()))
    np.savez_compressed(HERE / f"{out_prefix}.npz", **arrays)
    json.dump(meta, open(HERE / f"{out_prefix}.json", "w"), indent=1)
    print(f"[golden] {out_prefix}: loss={meta['enc_loss']:.6f} detail={meta['detail']} min_gap={meta['min_gap']:.3g}")


def encode_fixture(name, wseed, eseed, bseed, shapes, out_prefix):
    """Inference: the reference's Model.encode
    (vqvae.py:45-52 -> layers_vq.py:236-252, the path of bin/extract_bnf.py:
    47-69) in eval mode on a trained-shape codebook, at odd utterance lengths:
    the ids, the top-2 relative distance gap of every frame (computed from the
    reference encoder's z with the reference's distance formula), and the
    reference's Model.decode of those ids (vqvae.py:55-60)."""
    cfg = load_cfg(name)
    sd = seeded_state_dict(cfg, wseed)
    rng = np.random.Generator(np.random.PCG64(eseed))
    sd["quantizer.emb_init"] = torch.tensor(True)
    sd["quantizer.embeddings"] = torch.from_numpy(
        (rng.standard_normal((cfg["z_num"], cfg["z_dim"])) * 0.3).astype(np.float32))
    m = ref_model(cfg, sd)
    m.eval()
    arrays, meta = {}, dict(config=name, wseed=wseed, eseed=eseed, bseed=bseed, shapes=[list(s) for s in shapes],
                            cases=[])
    with torch.no_grad():
        for i, (B, T) in enumerate(shapes):
            x, y = seeded_batch(cfg, B, T, bseed + i)
            ids = m.encode(x)
            z = m.encoder(x)
            zf = z.transpose(1, 2).contiguous().view(-1, z.shape[1])
            E = m.quantizer.embeddings
            dist = (torch.sum(zf.pow(2), dim=1, keepdim=True) + torch.sum(E.pow(2), dim=1)) - 2 * torch.matmul(zf, E.t())
            top2 = torch.topk(dist, 2, dim=1, largest=False).values
            gap = (top2[:, 1] - top2[:, 0]) / top2[:, 1].abs().clamp_min(1e-30)
            assert torch.equal(torch.argmin(dist, dim=1), ids.reshape(-1))
            xhat = m.decode((ids, y))
            arrays[f"ids{i}"] = ids.reshape(-1).numpy().astype(np.int16)
            arrays[f"gap{i}"] = gap.numpy().astype(np.float32)
            arrays[f"xhat_head{i}"] = xhat.reshape(-1)[:256].numpy().astype(np.float32)
            meta["cases"].append(dict(B=B, T=T, xhat=summarize(xhat), n_gap_lt_1e4=int((gap < 1e-4).sum()),
                                      min_gap=float(gap.min())))
    np.savez_compressed(HERE / f"{out_prefix}.npz", **arrays)
    json.dump(meta, open(HERE / f"{out_prefix}.json", "w"), indent=1)
    print(f"[golden] {out_prefix}: " + ", ".join(f"{c['B']}x{c['T']} min_gap={c['min_gap']:.3g} "
                                                 f"<1e-4: {c['n_gap_lt_1e4']}" for c in meta["cases"]))


def vq_tile_fixture(seed, out_prefix):
    """N < K: init_emb and update_emb tile z with N(0, (0.01/sqrt(D))^2) noise."""
    from vae_npvc.model.layers_vq import EMAVectorQuantizer
    K, D, B, T = 512, 128, 1, 96
    rng = np.random.Generator(np.random.PCG64(seed))
    z = torch.from_numpy(rng.standard_normal((B, D, T)).astype(np.float32))
    q = EMAVectorQuantizer(K, D, 0.9, reduction="frame_mean")
    q.train()
    torch.manual_seed(seed + 1)
    zq, _, enc_loss, detail = q(z)  # first call: init_emb + update_emb
    arrays = dict(emb_row_norm=q.embeddings.norm(dim=1).numpy().astype(np.float32),
                  emb_elem=q.emb_elem.numpy().astype(np.float32))
    meta = dict(K=K, D=D, B=B, T=T, seed=seed, torch_seed=seed + 1, enc_loss=float(enc_loss),
                detail={k: float(v) for k, v in detail.items()}, embeddings=summarize(q.embeddings),
                emb_sum=summarize(q.emb_sum))
    np.savez_compressed(HERE / f"{out_prefix}.npz", **arrays)
    json.dump(meta, open(HERE / f"{out_prefix}.json", "w"), indent=1)
    print(f"[golden] {out_prefix}: {meta['detail']}")


def jitter_fixture():
    from vae_npvc.model.layers_vq import Jitter
    out = {}
    for p, T, seed in [(0.12, 256, 5), (0.12, 64, 6), (0.5, 33, 7)]:
        j = Jitter(probability=p)
        j.train()
        np.random.seed(seed)
        x = torch.arange(T, dtype=torch.float32).view(1, 1, T).repeat(2, 3, 1)
        y = j(x.clone())
        out[f"{p}_{T}_{seed}"] = dict(p=p, T=T, seed=seed, src=[int(v) for v in y[0, 0].tolist()],
                                      next_uniform=float(np.random.random_sample()))
    json.dump(out, open(HERE / "jitter.json", "w"), indent=1)
    print("[golden] jitter:", {k: sum(a != b for a, b in zip(v["src"], range(v["T"]))) for k, v in out.items()})


def structure_fixture():
    from vae_npvc.model.vqvae import Model
    out = {}
    for name in CFGS:
        cfg = load_cfg(name)
        m = Model(cfg)
        out[name] = dict(state_dict=[[k, list(v.shape)] for k, v in m.state_dict().items()],
                         parameters=[k for k, _ in m.named_parameters()],
                         n_params=int(sum(p.numel() for p in m.parameters())))
        ours = [[k, list(s)] for k, s in layer_specs(cfg)]
        assert [k for k, _ in ours] == out[name]["parameters"], "oracle parameter order != reference"
        ref_shapes = dict((k, s) for k, s in out[name]["state_dict"])
        for k, s in ours + [[k, list(s)] for k, s in buffer_specs(cfg)]:
            assert ref_shapes[k] == list(s), (k, ref_shapes[k], s)
    json.dump(out, open(HERE / "structure.json", "w"), indent=1)
    print("[golden] structure:", {k: v["n_params"] for k, v in out.items()})


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    if "--only-radam" in sys.argv:  # the §8f row-4 optimizer: 8 steps cross RAdam's N_sma >= 5 switch at step 6
        step_fixture("vcc20_radam", B=4, T=128, steps=8, wseed=1201, bseed=2201, tseed=3201, nseed=4201,
                     out_prefix="step_vcc20_radam")
        sys.exit(0)
    if "--only-multi" in sys.argv:  # the §8f row-4 general topology
        for i, name in enumerate(MULTI):
            step_fixture(name, B=4, T=128, steps=3, wseed=1301 + i, bseed=2301 + i, tseed=3301 + i, nseed=4301 + i,
                         out_prefix=f"step_{name}")
        sys.exit(0)
    if "--only-nown" in sys.argv:  # use_weight_norm: false (vqvae.py:179-180,290-293), plain convs throughout
        for i, name in enumerate(NOWN):
            step_fixture(name, B=4, T=128, steps=3, wseed=1401 + i, bseed=2401 + i, tseed=3401 + i, nseed=4401 + i,
                         out_prefix=f"step_{name}")
        sys.exit(0)
    if "--only-zdim" in sys.argv:  # codebook widths 64 / 256 (EMA and straight-through quantizers)
        for i, name in enumerate(ZDIM):
            step_fixture(name, B=4, T=128, steps=3, wseed=1501 + i, bseed=2501 + i, tseed=3501 + i, nseed=4501 + i,
                         out_prefix=f"step_{name}")
        sys.exit(0)
    if "--only-big" in sys.argv:  # config 3's data-parallel global batch (8 x 64 x 256)
        step_fixture("vcc20", B=512, T=256, steps=2, wseed=1004, bseed=2004, tseed=3004, nseed=4004,
                     out_prefix="full_step_vcc20_b512", compact=True)
        sys.exit(0)
    if "--only-encode" in sys.argv:  # §8f row 3: Model.encode / decode in eval mode (round 6)
        for i, name in enumerate(CFGS):
            encode_fixture(name, wseed=1601 + i, eseed=1701 + i, bseed=1801 + 10 * i,
                           shapes=[(2, 333), (1, 129), (3, 97)], out_prefix=f"encode_{name}")
        sys.exit(0)
    if "--only-plain" in sys.argv:  # just the §8f row-1 fixtures
        for i, name in enumerate(VARIANTS):
            step_fixture(name, B=4, T=128, steps=3, wseed=1101 + i, bseed=2101 + i, tseed=3101 + i,
                         nseed=4101 + i, out_prefix=f"step_{name}")
        sys.exit(0)
    structure_fixture()
    jitter_fixture()
    step_fixture("vcc20", B=4, T=128, steps=3, wseed=1001, bseed=2001, tseed=3001, nseed=4001, out_prefix="step_vcc20")
    step_fixture("aishell3", B=4, T=128, steps=3, wseed=1002, bseed=2002, tseed=3002, nseed=4002,
                 out_prefix="step_aishell3")
    for i, name in enumerate(VARIANTS):
        step_fixture(name, B=4, T=128, steps=3, wseed=1101 + i, bseed=2101 + i, tseed=3101 + i, nseed=4101 + i,
                     out_prefix=f"step_{name}")
    for i, name in enumerate(MULTI):
        step_fixture(name, B=4, T=128, steps=3, wseed=1301 + i, bseed=2301 + i, tseed=3301 + i, nseed=4301 + i,
                     out_prefix=f"step_{name}")
    step_fixture("vcc20_radam", B=4, T=128, steps=8, wseed=1201, bseed=2201, tseed=3201, nseed=4201,
                 out_prefix="step_vcc20_radam")
    for i, name in enumerate(NOWN):
        step_fixture(name, B=4, T=128, steps=3, wseed=1401 + i, bseed=2401 + i, tseed=3401 + i, nseed=4401 + i,
                     out_prefix=f"step_{name}")
    for i, name in enumerate(ZDIM):
        step_fixture(name, B=4, T=128, steps=3, wseed=1501 + i, bseed=2501 + i, tseed=3501 + i, nseed=4501 + i,
                     out_prefix=f"step_{name}")
    for K in (128, 512, 1024):
        vq_fixture(K, 64, 256, 5000 + K, f"vq_K{K}")
    vq_tile_fixture(6001, "vq_tile")
    if "--no-full" not in sys.argv:
        step_fixture("vcc20", B=64, T=256, steps=2, wseed=1003, bseed=2003, tseed=3003, nseed=4003,
                     out_prefix="full_step_vcc20")
