"""Inference drivers on the MI355X: Decoder.decode
(decoder/basic.py:41-75) and bin/extract_bnf (bin/extract_bnf.py:22-67)
through Model.encode/decode on libvqx, against the CPU oracle on the same
weights and features, with real Kaldi archives in and out."""
import numpy as np
import pytest
import torch

from helpers import assert_ids_near_tie_exact, cfg_of, load_fixture, oracle_encode_gaps

pytestmark = pytest.mark.gpu


def _setup(tmp_path, lengths=(333, 256, 129)):
    from oracle.vqvae_cpu import OracleVQVAE, seeded_state_dict
    from vae_npvc_amd.dataset import kaldi_io as K
    cfg = cfg_of("vcc20", compute_dtype="fp32")
    sd = seeded_state_dict(cfg, 91)
    rng = np.random.Generator(np.random.PCG64(3))
    sd["quantizer.emb_init"] = torch.tensor(True)
    sd["quantizer.embeddings"] = torch.from_numpy(rng.standard_normal((512, 128)).astype(np.float32) * 0.3)
    ckpt = tmp_path / "ckpt.pt"
    torch.save({"model": sd, "iteration": 12}, ckpt)
    data = tmp_path / "eval"
    data.mkdir()
    feats = {}
    with K.WriteHelper(f"ark,scp:{data}/feats.ark,{data}/feats.scp") as w:
        for i, n in enumerate(lengths):
            feats[f"src_{i}"] = rng.standard_normal((n, 80)).astype(np.float32)
            w[f"src_{i}"] = feats[f"src_{i}"]
    with open(data / "trials", "w") as f:
        for i, u in enumerate(feats):
            f.write(f"{u} TGT{i}\n")
    with open(data / "spk2spk_id", "w") as f:
        for i in range(len(feats)):
            f.write(f"TGT{i} {(i * 37) % 117}\n")
    orc = OracleVQVAE(cfg, sd)
    orc.training = False
    return cfg, ckpt, data, feats, orc


@pytest.mark.parametrize("compress", [False, True])
def test_decoder_converts_trials_like_oracle(tmp_path, compress):
    from vae_npvc_amd.dataset import kaldi_io as K
    from vae_npvc_amd.decoder.basic import Decoder
    cfg, ckpt, data, feats, orc = _setup(tmp_path)
    dec = Decoder(cfg)
    assert dec.load_checkpoint(str(ckpt)) == 12
    out = tmp_path / "out"
    out.mkdir()
    dec.decode(data, out, compress=compress)
    got = dict(K.ReadHelper(f"scp:{out}/feats.scp"))
    assert list(got) == list(feats)
    for i, (utt, x) in enumerate(feats.items()):
        xin = torch.from_numpy(x.T.copy()).unsqueeze(0)
        y = torch.tensor([[(i * 37) % 117]])
        with torch.no_grad():
            ref = orc.decode(orc.encode(xin), y)[0].T.numpy()
        assert got[utt].shape == ref.shape == (x.shape[0], 80)
        err = np.linalg.norm(got[utt] - ref) / np.linalg.norm(ref)
        assert err < (5e-3 if compress else 1e-4), (utt, err)


def test_extract_bnf_ids_match_oracle(tmp_path):
    import yaml
    from vae_npvc_amd.bin.extract_bnf import main
    from vae_npvc_amd.dataset import kaldi_io as K
    cfg, ckpt, data, feats, orc = _setup(tmp_path)
    conf = tmp_path / "conf.yaml"
    conf.write_text(yaml.safe_dump(cfg))
    with torch.no_grad():
        ref, gaps = {}, {}
        for u, x in feats.items():
            ref[u], gaps[u] = oracle_encode_gaps(orc, torch.from_numpy(x.T.copy()).unsqueeze(0))
    n = main(["-c", str(conf), "--model_path", str(ckpt), "--bnf_kind", "id", f"scp:{data}/feats.scp",
              str(tmp_path / "id.txt")])
    assert n == len(feats)
    for line in open(tmp_path / "id.txt"):
        utt, toks = line.split()
        ids = np.array([int(t) for t in toks.strip("<>").split("><")])
        assert ids.shape == ref[utt].shape, utt
        assert_ids_near_tie_exact(ids, ref[utt], gaps[utt], utt)  # every mismatch at an oracle near-tie
    main(["-c", str(conf), "--model_path", str(ckpt), "--bnf_kind", "csid", "--output_txt", "false",
          f"ark:{data}/feats.ark", f"ark,scp:{tmp_path}/cs.ark,{tmp_path}/cs.scp"])
    got = dict(K.ReadHelper(f"scp:{tmp_path}/cs.scp"))
    ids_txt = {}
    for line in open(tmp_path / "id.txt"):
        utt, toks = line.split()
        ids_txt[utt] = np.array([int(t) for t in toks.strip("<>").split("><")])
    for u in ref:
        # csid = unique_consecutive of this run's own ids (extract_bnf.py:59), exactly
        own = ids_txt[u]
        assert np.array_equal(got[u], own[np.concatenate([[True], own[1:] != own[:-1]])]), u


@pytest.mark.parametrize("name", ["vcc20", "vcc20_multi"])
def test_remove_weight_norm_keeps_inference(name):
    """Model.remove_weight_norm (vqvae.py:93-103) on a trained-shape model, with
    the strided resampling convs of the general topology: the eval forward,
    Model.encode and Model.infer after removal equal those before it (the
    packed weights go from g*v/||v|| computed on the GPU to the baked plain
    weights), and both match the oracle."""
    from oracle.vqvae_cpu import OracleVQVAE, seeded_batch, seeded_state_dict
    from tests.helpers import cfg_of, make_trainer
    cfg = cfg_of(name, compute_dtype="fp32")
    sd = seeded_state_dict(cfg, 77)
    sd["quantizer.emb_init"] = torch.tensor(True)
    g = torch.Generator().manual_seed(3)
    sd["quantizer.embeddings"] = torch.randn(cfg["z_num"], 128, generator=g) * 0.1
    tr = make_trainer(cfg, 77)
    m = tr.model
    m.load_state_dict(sd)
    m.eval()
    x, y = seeded_batch(cfg, 2, 128, 9)
    xd, yd = x.cuda(), y.cuda()
    with torch.no_grad():
        xh0 = m((xd, yd))[0].cpu()
        idx0 = m.encode(xd).cpu()
        m.remove_weight_norm()
        assert not any(n.endswith("weight_v") for n, _ in m.named_parameters())
        xh1 = m((xd, yd))[0].cpu()
        idx1 = m.encode(xd).cpu()
        inf1 = m.infer((xd, yd)).cpu()
    orc = OracleVQVAE(cfg, sd)
    orc.training = False
    with torch.no_grad():
        ref_idx, gap = oracle_encode_gaps(orc, x)
    assert_ids_near_tie_exact(idx0.numpy(), ref_idx, gap, "before removal")
    assert_ids_near_tie_exact(idx1.numpy(), ref_idx, gap, "after removal")
    scale = float(xh0.abs().max())
    assert float((xh1 - xh0).abs().max()) <= 1e-5 * scale
    assert float((inf1 - xh1).abs().max()) <= 1e-5 * scale


@pytest.mark.parametrize("name", ["vcc20", "aishell3"])
def test_encode_decode_match_reference_fixture(name):
    """Model.encode / Model.decode in eval mode against the REFERENCE's own
    outputs (tests/golden/encode_<cfg>, make_golden.py --only-encode:
    vqvae.py:45-60, the path of bin/extract_bnf.py:47-69) at odd lengths
    (2 x 333, 1 x 129, 3 x 97): every id equals the reference's except at the
    reference's own near-ties (top-2 relative gap < 1e-4), and the decode of
    the reference's ids matches its xhat within 1e-4 (fp32)."""
    import json
    from oracle.vqvae_cpu import seeded_batch, seeded_state_dict
    from vae_npvc_amd.model.vqvae import Model
    meta, arr = load_fixture(f"encode_{name}")
    cfg = cfg_of(name, compute_dtype="fp32")
    sd = seeded_state_dict(cfg, meta["wseed"])
    rng = np.random.Generator(np.random.PCG64(meta["eseed"]))
    sd["quantizer.emb_init"] = torch.tensor(True)
    sd["quantizer.embeddings"] = torch.from_numpy(
        (rng.standard_normal((cfg["z_num"], cfg["z_dim"])) * 0.3).astype(np.float32))
    m = Model(cfg)
    m.load_state_dict(sd)
    m = m.cuda().eval()
    flips = []
    with torch.no_grad():
        for i, c in enumerate(meta["cases"]):
            x, y = seeded_batch(cfg, c["B"], c["T"], meta["bseed"] + i)
            ids = m.encode(x.cuda()).cpu()
            assert tuple(ids.shape) == (c["B"], c["T"])
            flips.append(assert_ids_near_tie_exact(ids.numpy(), arr[f"ids{i}"], arr[f"gap{i}"], f"{c['B']}x{c['T']}"))
            ref_ids = torch.from_numpy(arr[f"ids{i}"].astype(np.int64)).view(c["B"], c["T"])
            xhat = m.decode((ref_ids.cuda(), y.cuda())).cpu().double()
            assert abs(float(xhat.norm()) - c["xhat"]["norm"]) <= 1e-4 * c["xhat"]["norm"], (i, float(xhat.norm()))
            head = torch.from_numpy(arr[f"xhat_head{i}"]).double()
            scale = float(head.abs().max())
            assert float((xhat.reshape(-1)[:256] - head).abs().max()) <= 1e-4 * scale, i
    print(json.dumps({"config": name, "id_flips_at_near_ties": flips}))
