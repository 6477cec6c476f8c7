"""Plugins for exercising vae_npvc_amd/bin/train.py without a GPU: a Dataset
whose items name their utterance index and a Trainer that records what each
rank was fed (the YAML `dataset_type` / `trainer_type` seams,
vae_npvc/bin/train.py:33-34,49-66)."""
import torch
import torch.distributed as dist


class Utts(torch.utils.data.Dataset):
    """Item i = (x (2, 4) filled with i, y = [i]): the (mel, T) / (1,) contract."""

    def __init__(self, data_dir, config, valid=False):
        self.n = config["n_valid"] if valid else config["n_utts"]

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return torch.full((2, 4), float(i)), torch.tensor([i])


class Trainer:
    def __init__(self, config):
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.iteration = 0
        self.seen = []      # (iteration, utterance ids of the batch)
        self.saved = []
        self.valids = 0

    def train_step(self, batch, iteration=None):
        x, y = batch
        self.iteration += 1
        self.seen.append((self.iteration, y.view(-1).tolist()))
        return self.iteration, {"Total": 10.0 * (self.rank + 1), "X like": float(self.rank + 1)}

    def valid(self, loader):
        self.valids += 1
        n = sum(len(b[1]) for b in loader)
        return {"X like": [1.0 / self.valids] * max(1, n)}

    def get_model_info(self):
        return "stub"

    def save_checkpoint(self, path):
        torch.save({"iteration": self.iteration, "rank": self.rank}, path)
        self.saved.append(str(path))

    def load_checkpoint(self, path):
        self.iteration = int(torch.load(path, weights_only=True)["iteration"])
        return self.iteration


class SynthMel(torch.utils.data.Dataset):
    """Seeded synthetic (mel (mel, T) f32, speaker (1,) int64) items -- the
    utt2mel_spk.py:42-74 contract without Kaldi archives."""

    def __init__(self, data_dir, config, valid=False):
        n = config["n_valid"] if valid else config["n_utts"]
        g = torch.Generator().manual_seed(2 if valid else 1)
        mel = config["encoder"]["in_channels"][0]
        T = config.get("crop_length", 256)
        self.x = torch.randn(n, mel, T, generator=g)
        self.y = torch.randint(0, config["y_num"], (n, 1), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], self.y[i]
