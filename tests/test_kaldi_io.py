"""Kaldi feature I/O and the training Dataset (SURVEY §8a row a-1, §8f rows
2-3), CPU only.

Parity: the reference reads features with kaldiio.load_mat
(dataset/utt2mel_spk.py:63) and writes them with kaldiio.WriteHelper
(decoder/basic.py:52-75).  Neither kaldiio nor Kaldi is in this image, so the
codec is pinned against blobs built here byte by byte from Kaldi's documented
CompressedMatrix layout and decoded by a scalar restatement of
Uint16ToFloat / CharToFloat (parity with Kaldi-written files: unpinned).
The Dataset is pinned against a line-by-line restatement of
utt2mel_spk.py:42-74 on the same global `random` stream.
"""
import random
import struct

import numpy as np
import pytest
import torch

from vae_npvc_amd.dataset import kaldi_io as K


def _scalar_cm1(min_value, rng, hdr, data, rows, cols):
    """Kaldi CompressedMatrix format 1 decode, one element at a time."""
    inc = np.float32(rng) * np.float32(1.0 / 65535.0)
    out = np.zeros((rows, cols), np.float32)
    for c in range(cols):
        p0, p25, p75, p100 = (np.float32(min_value) + inc * np.float32(h) for h in hdr[c])
        for r in range(rows):
            v = int(data[c * rows + r])
            if v <= 64:
                out[r, c] = p0 + (p25 - p0) * np.float32(v) * np.float32(1 / 64.0)
            elif v <= 192:
                out[r, c] = p25 + (p75 - p25) * np.float32(v - 64) * np.float32(1 / 128.0)
            else:
                out[r, c] = p75 + (p100 - p75) * np.float32(v - 192) * np.float32(1 / 63.0)
    return out


def test_cm1_handbuilt_blob_decodes_per_kaldi_layout(tmp_path):
    rows, cols = 7, 3
    min_value, rng = -2.5, 6.0
    hdr = [(0, 9000, 40000, 65535), (100, 200, 300, 400), (30000, 30001, 30002, 65000)]
    data = bytes((i * 37 + 11) % 256 for i in range(rows * cols))  # column-major on disk
    blob = b"CM " + struct.pack("<ffii", min_value, rng, rows, cols)
    blob += b"".join(struct.pack("<4H", *h) for h in hdr) + data
    ark = tmp_path / "cm.ark"
    ark.write_bytes(b"utt1 \x00B" + blob)
    got = K.load_mat(f"{ark}:5")
    ref = _scalar_cm1(min_value, rng, hdr, data, rows, cols)
    np.testing.assert_array_equal(got, ref)
    assert dict(K.ReadHelper(f"ark:{ark}"))["utt1"].shape == (rows, cols)


def test_cm2_cm3_handbuilt_blobs():
    rows, cols = 4, 5
    vals16 = np.arange(rows * cols, dtype=np.uint16) * 3000
    blob = b"CM2 " + struct.pack("<ffii", 1.0, 2.0, rows, cols) + vals16.astype("<u2").tobytes()
    got = K.decompress(blob)
    ref = np.float32(1.0) + np.float32(2.0) * np.float32(1 / 65535.0) * vals16.reshape(rows, cols).astype(np.float32)
    np.testing.assert_array_equal(got, ref)
    vals8 = (np.arange(rows * cols) * 13 % 256).astype(np.uint8)
    blob = b"CM3 " + struct.pack("<ffii", -1.0, 4.0, rows, cols) + vals8.tobytes()
    ref = np.float32(-1.0) + np.float32(4.0) * np.float32(1 / 255.0) * vals8.reshape(rows, cols).astype(np.float32)
    np.testing.assert_array_equal(K.decompress(blob), ref)


@pytest.mark.parametrize("rows", [1, 3, 6, 9, 300])
def test_compress_roundtrip_error_bounds(rows):
    rng = np.random.default_rng(rows)
    m = (rng.standard_normal((rows, 80)) * 3 + 1).astype(np.float32)
    span = float(m.max() - m.min()) or 1.0
    d2 = K.decompress(K.compress(m, K.K_TWO_BYTE_AUTO))
    assert np.abs(d2 - m).max() <= span / 65535.0 + 1e-6
    d3 = K.decompress(K.compress(m, K.K_ONE_BYTE_AUTO))
    assert np.abs(d3 - m).max() <= span / 255.0 * 0.51 + 1e-6
    d1 = K.decompress(K.compress(m, K.K_SPEECH_FEATURE))
    assert d1.shape == m.shape
    # one byte between column percentiles: error <= half a step of the widest interval
    assert np.abs(d1 - m).max() <= span / 63.0 + span / 65535.0 + 1e-5
    auto = K.compress(m, K.K_AUTO)
    assert auto.startswith(b"CM " if rows > 8 else b"CM2 ")


def test_ark_scp_roundtrip_ranges_and_int_vectors(tmp_path):
    rng = np.random.default_rng(0)
    mats = {f"utt{i}": rng.standard_normal((20 + 13 * i, 80)).astype(np.float32) for i in range(4)}
    with K.WriteHelper(f"ark,scp:{tmp_path}/f.ark,{tmp_path}/f.scp") as w:
        for k, v in mats.items():
            w[k] = v
        w["dbl"] = np.arange(12, dtype=np.float64).reshape(3, 4)
        w["ids"] = np.array([3, 1, 4, 1, 5], dtype=np.int64)
    scp = K.load_scp(tmp_path / "f.scp")
    for k, v in mats.items():
        np.testing.assert_array_equal(K.load_mat(scp[k]), v)
        np.testing.assert_array_equal(K.load_mat(scp[k] + "[5:9]"), v[5:10])
        np.testing.assert_array_equal(K.load_mat(scp[k] + "[2:3,10:19]"), v[2:4, 10:20])
    assert K.load_mat(scp["dbl"]).dtype == np.float64
    np.testing.assert_array_equal(K.load_mat(scp["ids"]), [3, 1, 4, 1, 5])
    keys = [k for k, _ in K.ReadHelper(f"ark:{tmp_path}/f.ark")]
    assert keys == list(mats) + ["dbl", "ids"]
    assert [k for k, _ in K.ReadHelper(f"scp:{tmp_path}/f.scp")] == keys
    with pytest.raises(ValueError):
        K.WriteHelper(f"scp:{tmp_path}/x.scp")


def _make_data_dir(root, lengths, mel=80, compression=None):
    rng = np.random.default_rng(5)
    mats = {}
    with K.WriteHelper(f"ark,scp:{root}/feats.ark,{root}/feats.scp", compression_method=compression) as w:
        for i, n in enumerate(lengths):
            utt = f"spk{i % 3}_utt{i}"
            mats[utt] = rng.standard_normal((n, mel)).astype(np.float32)
            w[utt] = mats[utt]
    with open(root / "utt2num_frames", "w") as f:
        for u, m in mats.items():
            f.write(f"{u} {m.shape[0]}\n")
    with open(root / "utt2spk_id", "w") as f:
        for i, u in enumerate(mats):
            f.write(f"{u} {i % 3 + 7}\n")
    return mats


def _reference_getitem(mats, utt2spk, index, crop_length, valid):
    """utt2mel_spk.py:42-74 restated on in-memory matrices (same random draws)."""
    utt, spk = utt2spk[index]
    feat_length = mats[utt].shape[0]
    if feat_length <= crop_length:
        s, e = 0, feat_length
    else:
        s = random.randint(0, feat_length - crop_length) if not valid else 0
        e = s + crop_length
    feat = torch.from_numpy(mats[utt][s:e].T.copy()).float()
    if feat_length < crop_length:
        feat = torch.nn.functional.pad(feat, (0, crop_length - feat_length))
    return feat, torch.tensor([int(spk)]).long()


@pytest.mark.parametrize("valid", [False, True])
def test_dataset_matches_reference_getitem(tmp_path, valid):
    from vae_npvc_amd.dataset.utt2mel_spk import Dataset
    lengths = [100, 256, 400, 257, 999]
    mats = _make_data_dir(tmp_path, lengths)
    cfg = {"crop_length": 256}
    ds = Dataset(tmp_path, cfg, valid=valid)
    assert len(ds) == len(lengths)
    utt2spk = [line.split() for line in open(tmp_path / "utt2spk_id")]
    for rep in range(3):
        random.seed(100 + rep)
        got = [ds[i] for i in range(len(ds))]
        random.seed(100 + rep)
        ref = [_reference_getitem(mats, utt2spk, i, 256, valid) for i in range(len(ds))]
        for (x, y), (xr, yr) in zip(got, ref):
            assert x.shape == (80, 256) and x.dtype == torch.float32
            assert torch.equal(x, xr)
            assert torch.equal(y, yr) and y.dtype == torch.int64
    assert torch.all(ds[0][0][:, 100:] == 0)  # zero padding of the short utterance


def test_dataset_compressed_features_and_collate(tmp_path):
    from vae_npvc_amd.dataset.utt2mel_spk import Dataset
    mats = _make_data_dir(tmp_path, [300, 260, 512, 256], compression=K.K_SPEECH_FEATURE)
    ds = Dataset(tmp_path, {"crop_length": 256, "valid_crop_length": 128}, valid=True)
    x, y = ds[2]
    ref = K.decompress(K.compress(mats["spk2_utt2"], K.K_SPEECH_FEATURE))[:128].T
    np.testing.assert_array_equal(x.numpy(), ref)
    loader = torch.utils.data.DataLoader(Dataset(tmp_path, {"crop_length": 256}), batch_size=4, shuffle=True,
                                         drop_last=True)
    xb, yb = next(iter(loader))
    assert xb.shape == (4, 80, 256) and yb.shape == (4, 1) and yb.dtype == torch.int64
