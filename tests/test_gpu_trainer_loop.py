"""The drop-in Trainer under the reference's own training loop (-m gpu).

`run_reference_loop` restates vae_npvc/bin/train.py:44-167 (seeding, trainer
construction through the YAML `trainer_type` string, checkpoint resume with
`iteration = load_checkpoint(path) + 1`, the DataLoader over the recipe's
Dataset, `iteration, loss_detail = trainer.train_step(batch,
iteration=iteration)`, per-log averaging, checkpoint + validation cadence,
the max_iter exit) with the training data replaced by an in-memory synthetic
dataset (no Kaldi archives or logging handlers).  The reference's script
cannot be imported on the GPU box (the reference never travels), so the loop
is restated line by line.
"""
from importlib import import_module

import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader, Dataset

from tests.helpers import cfg_of

pytestmark = pytest.mark.gpu


class SyntheticMel(Dataset):
    """(mel (80, T) f32, speaker id (1,) int64) items, the utt2mel_spk.py:42-74 contract."""

    def __init__(self, n, T, y_num, seed):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, 80, T, generator=g)
        self.y = torch.randint(0, y_num, (n, 1), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], self.y[i]


def run_reference_loop(config, checkpoint_path, output_dir, train_set, valid_set):
    """bin/train.py:24-167 minus I/O plumbing; returns what the loop observed."""
    trainer_type = config.get("trainer_type").split(":")
    max_iter = config.get("max_iter", 100000)
    iters_per_checkpoint = config.get("iters_per_checkpoint", 10000)
    iters_per_log = config.get("iters_per_log", 1000)
    check_loss_kind = config.get("check_loss_kind", "X like")
    seed = config.get("seed", 777)
    np.random.seed(seed)
    torch.manual_seed(seed)
    trainer_module = import_module(trainer_type[0], package=None)
    trainer_name = "Trainer" if len(trainer_type) < 2 else trainer_type[1]
    trainer = getattr(trainer_module, trainer_name)(config)
    iteration = 1
    if checkpoint_path is not None:
        iteration = trainer.load_checkpoint(checkpoint_path)
        iteration += 1
    train_loader = DataLoader(train_set, num_workers=0, shuffle=True, batch_size=config["batch_size"],
                              drop_last=True)
    valid_loader = DataLoader(valid_set, num_workers=0, shuffle=False, batch_size=config["batch_size"])
    seen, logs, ckpts, valids = [], [], [], []
    train_log = dict()
    best_loss = {check_loss_kind: np.inf}
    best_iter = 0
    while iteration <= max_iter:
        for i, batch in enumerate(train_loader):
            iteration, loss_detail = trainer.train_step(batch, iteration=iteration)
            seen.append(iteration)
            for key, val in loss_detail.items():
                train_log.setdefault(key, []).append(val)
            if iteration % iters_per_log == 0 and len(train_log.keys()) > 0:
                logs.append((iteration, {k: float(np.mean(v)) for k, v in train_log.items()}))
                train_log = dict()
            if iteration % iters_per_checkpoint == 0:
                path = output_dir / "iter.{}".format(iteration)
                trainer.save_checkpoint(path)
                ckpts.append(path)
            if iteration % iters_per_checkpoint == 0 and valid_loader is not None:
                loss_detail = trainer.valid(valid_loader)
                best_check_loss = np.mean(best_loss[check_loss_kind])
                check_loss = np.mean(loss_detail[check_loss_kind])
                if best_check_loss >= check_loss:
                    best_loss = loss_detail
                    best_iter = iteration
                valids.append((iteration, loss_detail))
            if iteration > max_iter:
                break
    return dict(seen=seen, logs=logs, ckpts=ckpts, valids=valids, best_iter=best_iter, trainer=trainer)


def test_reference_training_loop_advances_checkpoints_and_resumes(tmp_path):
    cfg = cfg_of("vcc20", compute_dtype="fp32", batch_size=2, max_iter=6, iters_per_log=2,
                 iters_per_checkpoint=3)
    train_set = SyntheticMel(8, 64, cfg["y_num"], 1)
    valid_set = SyntheticMel(2, 64, cfg["y_num"], 2)
    out = run_reference_loop(cfg, None, tmp_path, train_set, valid_set)
    # the loop advances; like the reference it exits after the first step past
    # max_iter (bin/train.py:123,166-168: 4 batches per epoch, steps 5-7 in epoch 2)
    assert out["seen"] == [1, 2, 3, 4, 5, 6, 7]
    assert [it for it, _ in out["logs"]] == [2, 4, 6]
    assert set(out["logs"][0][1]) == {"Total", "VQ loss", "X like", "entropy", "used_curr", "usage", "diff_emb"}
    assert [p.name for p in out["ckpts"]] == ["iter.3", "iter.6"]
    assert [it for it, _ in out["valids"]] == [3, 6]
    assert all(len(v["X like"]) == 1 for _, v in out["valids"])  # one validation batch of 2
    assert out["best_iter"] in (3, 6)
    ck = torch.load(out["ckpts"][0], map_location="cpu", weights_only=True)
    assert ck["iteration"] == 3 and set(ck) == {"model", "optimizer", "iteration"}
    # resume from iter.3: train.py passes load_checkpoint(...) + 1 and counts on
    res = run_reference_loop(dict(cfg, max_iter=7), out["ckpts"][0], tmp_path, train_set, valid_set)
    assert res["seen"] == [4, 5, 6, 7, 8]
    assert int(res["trainer"].engine.opt_step.item()) == 8  # optimizer state resumed with the weights


def test_train_entry_single_gpu_runs_the_reference_loop(tmp_path):
    """vae_npvc_amd/bin/train.py itself (world size 1: the reference's shuffled
    DataLoader) with the real Trainer: iterations 1..7 for max_iter 6,
    checkpoints iter.3 / iter.6 with the reference's keys, validation picks
    the best checkpoint, resume continues at checkpoint + 1."""
    import types

    import yaml
    from vae_npvc_amd.bin import train as entry
    cfg = cfg_of("vcc20", compute_dtype="fp32", batch_size=2, max_iter=6, iters_per_log=2,
                 iters_per_checkpoint=3, crop_length=64, num_jobs=0, n_utts=8, n_valid=2,
                 dataset_type="tests.ddp_stubs:SynthMel")
    path = tmp_path / "conf.yaml"
    yaml.safe_dump(cfg, open(path, "w"))
    args = types.SimpleNamespace(config=str(path), output_dir=str(tmp_path / "exp"), checkpoint=None,
                                 train_dir="unused", valid_dir="unused", backend=None)
    tr = entry.train(args)
    assert tr.iteration == 7
    exp = tmp_path / "exp"
    ck = torch.load(exp / "iter.6", map_location="cpu", weights_only=True)
    assert ck["iteration"] == 6 and set(ck) == {"model", "optimizer", "iteration"}
    assert (exp / "model.loss.best").exists()
    log = (exp / "train.log").read_text()
    assert [l.split("Iter ")[1].split(":")[0] for l in log.splitlines() if " Iter " in l] == ["2", "4", "6"]
    assert "Valid 3:" in log and "Valid 6:" in log
    yaml.safe_dump(dict(cfg, max_iter=7), open(path, "w"))
    args.checkpoint = str(exp / "iter.3")
    tr2 = entry.train(args)
    assert tr2.iteration == 8 and int(tr2.engine.opt_step.item()) == 8
