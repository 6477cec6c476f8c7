"""Pin the CPU oracle (oracle/vqvae_cpu.py) against golden vectors produced by
the reference itself (tests/golden/make_golden.py).  CPU only."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch
import yaml

from oracle.vqvae_cpu import OracleTrainer, layer_specs, seeded_batch, seeded_state_dict

GOLD = Path(__file__).resolve().parent / "golden"
CONF = Path(__file__).resolve().parent.parent / "vae_npvc_amd" / "conf"


def cfg_of(name):
    return yaml.safe_load(open(CONF / f"{name}.yaml"))


def helpers_cfg(name):
    from tests.helpers import cfg_of as hc
    return hc(name)


def load_fixture(prefix):
    meta = json.load(open(GOLD / f"{prefix}.json"))
    arr = dict(np.load(GOLD / f"{prefix}.npz", allow_pickle=False))
    return meta, arr


def close(a, b, rtol):
    return abs(a - b) <= rtol * max(abs(b), 1e-12)


def test_structure_matches_reference():
    st = json.load(open(GOLD / "structure.json"))
    for name in ("vcc20", "aishell3"):
        cfg = cfg_of(name)
        assert [k for k, _ in layer_specs(cfg)] == st[name]["parameters"]
        n = sum(int(np.prod(s)) for _, s in layer_specs(cfg))
        assert n == st[name]["n_params"]


FIXTURE_CFG = {"step_vcc20": ("vcc20", {}), "step_aishell3": ("aishell3", {}),
               "step_vcc20_radam": ("vcc20", {"optim_type": "RAdam"}), "step_vcc20_multi": ("vcc20_multi", {}),
               "step_vcc20_nown": ("vcc20_nown", {}), "step_vcc20_multi_nown": ("vcc20_multi_nown", {}),
               "step_vcc20_z64": ("vcc20_z64", {}), "step_vcc20_z256": ("vcc20_z256", {})}


@pytest.mark.parametrize("prefix", list(FIXTURE_CFG))
def test_oracle_train_steps_match_reference(prefix):
    """Adam (3 steps) and RAdam (8 steps: the rectified update starts at step 6,
    trainer/radam.py:53-59) against the reference run; step_vcc20_multi is the
    general Encoder/Decoder topology (two stages with strided resampling,
    dilation, stack_layers 2, decoder kernel 5) with EMA and jitter."""
    meta, arr = load_fixture(prefix)
    base, over = FIXTURE_CFG[prefix]
    cfg = dict(helpers_cfg(base), **over)
    torch.set_num_threads(4)
    tr = OracleTrainer(cfg, seeded_state_dict(cfg, meta["wseed"]))
    torch.manual_seed(meta["tseed"])
    np.random.seed(meta["nseed"])
    for s in range(meta["steps"]):
        batch = seeded_batch(cfg, meta["B"], meta["T"], meta["bseed"] + s)
        _, detail = tr.train_step(batch, keep_grads=(s == 0))
        ref = meta["detail"][s]
        for k, v in ref.items():
            rt = 1e-4 if k != "diff_emb" else 1e-3
            assert close(detail[k], v, rt), (s, k, detail[k], v)
        idx = tr.model.last["idx"].numpy()
        gap = arr[f"gap{s}"]
        mism = idx != arr[f"idx{s}"]
        # any disagreement must sit on a near-tie of the reference distances
        assert (gap[mism] < 1e-4).all(), (s, int(mism.sum()))
        assert mism.mean() < 0.01
        np.testing.assert_allclose(tr.model.emb_elem.numpy(), arr[f"emb_elem{s}"], rtol=1e-5, atol=1e-6)
        assert close(float(tr.model.embeddings.double().norm()), meta[f"embeddings{s}"]["norm"], 1e-4)
        if s == 0:
            np.testing.assert_allclose(tr.last_xhat[:, :, :16].numpy(), arr["xhat0_slice"], rtol=1e-3, atol=1e-3)
            for k, g in tr.grads.items():
                gn = float(g.double().norm())
                assert close(gn, meta["grads"][k]["norm"], 2e-3) or abs(gn - meta["grads"][k]["norm"]) < 1e-8, k
    for k, p in tr.model.params.items():
        assert close(float(p.detach().double().norm()), meta["params_after"][k]["norm"], 1e-4), k


PLAIN = {"vcc20_plain": ("vcc20", {"use_ema": False}),
         "vcc20_plain_nonorm": ("vcc20", {"use_ema": False, "embed_norm": False}),
         "aishell3_plain": ("aishell3", {"use_ema": False}),
         "vcc20_multi_plain": ("vcc20_multi_plain", {}),
         "vcc20_z64_plain": ("vcc20_z64_plain", {}), "vcc20_z256_plain": ("vcc20_z256_plain", {})}


def plain_cfg(name):
    base, over = PLAIN[name]
    return dict(helpers_cfg(base), **over)


@pytest.mark.parametrize("name", list(PLAIN))
def test_oracle_plain_vq_steps_match_reference(name):
    """Straight-through VectorQuantizer (use_ema: false):
    losses, perplexity, step-0 gradients (incl. the codebook parameter) and
    parameters after 3 Adam steps vs the reference run."""
    meta, arr = load_fixture(f"step_{name}")
    cfg = plain_cfg(name)
    torch.set_num_threads(4)
    tr = OracleTrainer(cfg, seeded_state_dict(cfg, meta["wseed"]))
    torch.manual_seed(meta["tseed"])
    np.random.seed(meta["nseed"])
    for s in range(meta["steps"]):
        batch = seeded_batch(cfg, meta["B"], meta["T"], meta["bseed"] + s)
        _, detail = tr.train_step(batch, keep_grads=(s == 0))
        ref = meta["detail"][s]
        assert set(detail) == set(ref)
        for k, v in ref.items():
            assert close(detail[k], v, 1e-4), (s, k, detail[k], v)
        if s == 0:
            np.testing.assert_allclose(tr.last_xhat[:, :, :16].numpy(), arr["xhat0_slice"], rtol=1e-3, atol=1e-3)
            for k, g in tr.grads.items():
                gn = float(g.double().norm())
                assert close(gn, meta["grads"][k]["norm"], 2e-3) or abs(gn - meta["grads"][k]["norm"]) < 1e-8, k
    for k, p in tr.model.params.items():
        assert close(float(p.detach().double().norm()), meta["params_after"][k]["norm"], 1e-4), k


@pytest.mark.parametrize("K", [128, 512, 1024])
def test_oracle_vq_matches_reference(K):
    from oracle.vqvae_cpu import OracleVQVAE
    meta, arr = load_fixture(f"vq_K{K}")
    cfg = cfg_of("vcc20")
    cfg = dict(cfg, z_num=K)
    rng = np.random.Generator(np.random.PCG64(meta["seed"]))
    D = 128
    z = torch.from_numpy(rng.standard_normal((meta["B"], D, meta["T"])).astype(np.float32))
    E = torch.from_numpy(rng.standard_normal((K, D)).astype(np.float32))
    emb_sum = torch.from_numpy((1.5 * rng.standard_normal((K, D))).astype(np.float32))
    emb_elem = torch.from_numpy(rng.uniform(0.5, 3.0, size=(K,)).astype(np.float32))
    sd = seeded_state_dict(cfg, 1)
    sd["quantizer.emb_init"] = torch.tensor(True)
    sd["quantizer.embeddings"], sd["quantizer.emb_sum"], sd["quantizer.emb_elem"] = E, emb_sum, emb_elem
    m = OracleVQVAE(cfg, sd)
    idx_eval = torch.argmin(m.distances(z.transpose(1, 2).reshape(-1, D), E), 1).numpy()
    assert (idx_eval == arr["idx_eval"]).all()
    torch.manual_seed(meta["torch_seed"])
    zq, _, enc_loss, detail = m.quantize(z)
    assert (m.last["idx"].numpy() == arr["idx"]).all()
    assert close(float(enc_loss), meta["enc_loss"], 1e-5)
    for k, v in meta["detail"].items():
        assert close(detail[k], v, 1e-5), (k, detail[k], v)
    np.testing.assert_allclose(m.emb_elem.numpy(), arr["emb_elem"], rtol=1e-6)
    np.testing.assert_allclose(m.embeddings.norm(dim=1).numpy(), arr["emb_row_norm"], rtol=1e-5)


def test_oracle_vq_tile_path():
    from oracle.vqvae_cpu import OracleVQVAE
    meta, arr = load_fixture("vq_tile")
    cfg = dict(cfg_of("vcc20"), z_num=meta["K"])
    rng = np.random.Generator(np.random.PCG64(meta["seed"]))
    z = torch.from_numpy(rng.standard_normal((meta["B"], meta["D"], meta["T"])).astype(np.float32))
    m = OracleVQVAE(cfg, seeded_state_dict(cfg, 1))
    torch.manual_seed(meta["torch_seed"])
    _, _, enc_loss, detail = m.quantize(z)
    assert close(float(enc_loss), meta["enc_loss"], 1e-5)
    for k, v in meta["detail"].items():
        assert close(detail[k], v, 1e-5), k
    np.testing.assert_allclose(m.embeddings.norm(dim=1).numpy(), arr["emb_row_norm"], rtol=1e-5)


def test_oracle_jitter_map_matches_reference():
    from oracle.vqvae_cpu import OracleVQVAE
    fx = json.load(open(GOLD / "jitter.json"))
    for v in fx.values():
        m = OracleVQVAE.__new__(OracleVQVAE)
        m.jitter_p, m.training = v["p"], True
        np.random.seed(v["seed"])
        x = torch.arange(v["T"], dtype=torch.float32).view(1, 1, -1).repeat(2, 3, 1)
        y = m.jitter(x.clone())
        assert [int(t) for t in y[0, 0].tolist()] == v["src"]
        assert np.random.random_sample() == v["next_uniform"]


@pytest.mark.slow
def test_oracle_full_size_step():
    meta, arr = load_fixture("full_step_vcc20")
    cfg = cfg_of(meta["config"])
    torch.set_num_threads(8)
    tr = OracleTrainer(cfg, seeded_state_dict(cfg, meta["wseed"]))
    torch.manual_seed(meta["tseed"])
    np.random.seed(meta["nseed"])
    for s in range(meta["steps"]):
        batch = seeded_batch(cfg, meta["B"], meta["T"], meta["bseed"] + s)
        _, detail = tr.train_step(batch)
        for k, v in meta["detail"][s].items():
            assert close(detail[k], v, 1e-3), (s, k, detail[k], v)
        mism = tr.model.last["idx"].numpy() != arr[f"idx{s}"]
        assert mism.mean() < 0.01
