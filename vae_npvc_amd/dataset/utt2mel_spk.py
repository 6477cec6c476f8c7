"""Training batches for the VQ-VAE step: the reference's
`vae_npvc.dataset.utt2mel_spk.Dataset` (dataset/utt2mel_spk.py:22-77) on this
package's Kaldi reader (kaldi_io.load_mat replaces kaldiio.load_mat).

Per item: a random crop of `train_crop_length` (default `crop_length`, 256)
frames of the utterance's (T, mel) matrix read by inclusive row range, zero
padding at the end when shorter (:56-70), transposed to (mel, T) fp32, and
the speaker id as a (1,) int64 tensor (:72).  Validation crops start at 0.
`random.randint` on Python's global generator draws the crop start exactly as
the reference does, so a seeded loader yields the reference's crops.
Default torch collation gives x (B, mel, T) and y (B, 1), the batch contract
of Trainer.train_step (trainer/basic.py:55-79).
"""
import random
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

from .kaldi_io import load_mat


def load_dict_data(data_file):
    """{rec: data} of a two-column Kaldi table (utt2mel_spk.py:11-14)."""
    lines = [line.strip().split(None, 1) for line in open(data_file)]
    return {x[0]: x[1] for x in lines if x}


def load_list_data(data_file):
    """[[rec, data...]] of a whitespace table (utt2mel_spk.py:16-18)."""
    return [line.strip().split() for line in open(data_file) if line.strip()]


class Dataset(torch.utils.data.Dataset):
    """feats.scp + utt2num_frames + utt2spk_id of one data directory."""

    def __init__(self, data_dir, config, valid=False):
        crop_length = config.get("crop_length", 256)
        key = "valid_crop_length" if valid else "train_crop_length"
        self.crop_length = config.get(key, crop_length)
        self.valid = valid
        data_dir = Path(data_dir)
        self.feats_scp = load_dict_data(data_dir / "feats.scp")
        self.utt2num_frames = load_dict_data(data_dir / "utt2num_frames")
        self.utt2spks = load_list_data(data_dir / "utt2spk_id")
        self.num_data = len(self.utt2spks)

    def crop_window(self, feat_length):
        """(start, end) frames of the crop (utt2mel_spk.py:50-56)."""
        if feat_length <= self.crop_length:
            return 0, feat_length
        max_feat_start = feat_length - self.crop_length
        start = random.randint(0, max_feat_start) if not self.valid else 0
        return start, start + self.crop_length

    def __getitem__(self, index):
        utt, spk = self.utt2spks[index]
        feat_length = int(self.utt2num_frames[utt])
        start, end = self.crop_window(feat_length)
        feat = np.array(load_mat("{}[{}:{}]".format(self.feats_scp[utt], start, end - 1)))  # (T, mel)
        feat = torch.from_numpy(feat.T).float()                                           # (mel, T)
        if feat_length < self.crop_length:
            feat = F.pad(feat, (0, self.crop_length - feat_length)).data
        return feat, torch.tensor([int(spk)]).long()

    def __len__(self):
        return self.num_data
