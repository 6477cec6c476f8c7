#!/usr/bin/env python3
"""Training entry, single GPU or data parallel (one process per GPU).

Restates vae_npvc/bin/train.py:24-204 -- YAML config, identical seeding,
`trainer_type` / `dataset_type` plugins through importlib, checkpoint resume
at `load_checkpoint(path) + 1`, the per-log averaging, checkpoint and
validation cadence, the best-model copy -- and adds what data parallelism
needs:

* started by `torch.distributed.run` (WORLD_SIZE > 1 in the environment), the
  process group is initialised from torchrun's env before any other GPU call
  (backend "nccl" = RCCL over xGMI when GPUs are visible, "gloo" otherwise)
  and the process takes GPU LOCAL_RANK; the Trainer then all-reduces
  gradients and EMA statistics (vae_npvc_amd/trainer/basic.py, parallel/ddp.py);
* the utterances are sharded with `ShardSampler` (dataset/sampler.py):
  disjoint per-rank shares of one per-epoch permutation, equal counts, so
  every rank runs the same iterations;
* `batch_size` (`train_batch_size`) is per rank, as BASELINE config 3 counts
  it (64 per GPU, global 512 on 8 GPUs); a `global_batch_size` key instead
  divides over the ranks;
* rank 0 alone writes the log, the checkpoints and the best-model copy and
  runs validation; the logged training means are averaged over the ranks once
  per log interval (one small all-reduce), the others wait at a barrier after
  each checkpoint.

At world size 1 the loop is the reference's: a shuffled DataLoader drawing
from the global torch generator.  One deliberate fix: when no validation ever
ran, the reference copies the nonexistent `iter.0` and crashes
(bin/train.py:173); here the copy is skipped with a log line.

    python -m vae_npvc_amd.bin.train -c conf.yaml --output_dir exp --train_dir data/train [--valid_dir ...]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m vae_npvc_amd.bin.train ...
"""
import datetime
import logging
import os
from importlib import import_module
from pathlib import Path
from shutil import copyfile

import numpy as np
import torch
import torch.distributed as dist
from torch.utils.data import DataLoader

from ..dataset.sampler import ShardSampler


DIST_TIMEOUT_S = 7200  # multi-rank default: rank 0's checkpoint validation while the others wait


def setup_distributed(backend=None, timeout_s=None):
    """Initialise the process group from torchrun's environment (before any
    other GPU call) and select GPU LOCAL_RANK.  Returns (world, rank, backend)
    -- (1, 0, None) when not launched with more than one process.
    `timeout_s` (config key `dist_timeout_s`) bounds every collective wait,
    e.g. the other ranks' barrier while rank 0 validates at a checkpoint;
    None keeps torch's default."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 1, 0, None
    if dist.is_initialized():
        return dist.get_world_size(), dist.get_rank(), dist.get_backend()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.device_count() > 0 else "gloo"  # device_count() does not initialise HIP
    kw = {} if timeout_s is None else dict(timeout=datetime.timedelta(seconds=float(timeout_s)))
    if backend == "nccl":
        dev = torch.device("cuda", local)
        dist.init_process_group("nccl", device_id=dev, **kw)
        torch.cuda.set_device(dev)
    else:
        dist.init_process_group(backend, **kw)
    return world, rank, backend


def _plugin(spec, default_name):
    parts = spec.split(":")
    return getattr(import_module(parts[0], package=None), default_name if len(parts) < 2 else parts[1])


def _logger(output_dir, rank):
    logger = logging.getLogger("logger")
    logger.setLevel(logging.INFO)
    for h in list(logger.handlers):  # a second train() in one process (tests) starts clean
        logger.removeHandler(h)
        h.close()
    if rank != 0:
        logger.addHandler(logging.NullHandler())
        logger.propagate = False
        return logger
    fmt = logging.Formatter("%(asctime)s %(message)s", datefmt="%m-%d %H:%M:%S")
    for h in (logging.StreamHandler(), logging.FileHandler(filename=str(output_dir / "train.log"))):
        h.setFormatter(fmt)
        logger.addHandler(h)
    return logger


def _ranks_mean(train_log, backend):
    """{key: mean over this rank's steps} averaged over the ranks (equal step
    counts and per-rank batches: the global-batch mean).  Keys in sorted
    order so every rank packs the same vector."""
    keys = sorted(train_log)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    v = torch.tensor([float(np.mean(train_log[k])) for k in keys], dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.SUM)
    v = (v / dist.get_world_size()).cpu().tolist()
    return dict(zip(keys, v))


def train(args):
    import yaml
    config = yaml.safe_load(open(args.config))  # host only: the process group comes before any GPU call
    # rank 0 alone validates at a checkpoint while the others wait in a barrier:
    # a long validation set needs more than torch's default collective timeout
    # (about 10 min for NCCL), so multi-rank runs default to DIST_TIMEOUT_S
    # unless the config sets dist_timeout_s (null keeps torch's default)
    timeout_s = config.get("dist_timeout_s", DIST_TIMEOUT_S if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None)
    world, rank, backend = setup_distributed(getattr(args, "backend", None), timeout_s)
    ddp = world > 1
    output_dir = args.output_dir
    checkpoint_path = args.checkpoint
    train_dir = args.train_dir
    valid_dir = args.valid_dir

    trainer_type = config.get("trainer_type", "vae_npvc_amd.trainer.basic:Trainer")
    dataset_type = config.get("dataset_type", "vae_npvc_amd.dataset.utt2mel_spk:Dataset")
    max_iter = config.get("max_iter", 100000)
    iters_per_checkpoint = config.get("iters_per_checkpoint", 10000)
    iters_per_log = config.get("iters_per_log", 1000)
    check_loss_kind = config.get("check_loss_kind", "X like")
    num_jobs = config.get("num_jobs", 8)
    seed = config.get("seed", 777)

    # identical on every rank: the EMA codebook's randperm and the jitter map
    # are drawn from these streams and must agree across ranks
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)

    trainer = _plugin(trainer_type, "Trainer")(config)

    iteration = 1
    if checkpoint_path is not None:
        iteration = trainer.load_checkpoint(checkpoint_path)
        iteration += 1

    dataset_module = import_module(dataset_type.split(":")[0], package=None)
    Dataset = _plugin(dataset_type, "Dataset")
    collate_fn = getattr(dataset_module, "collate", None)
    batch_size = config.get("train_batch_size", config.get("batch_size", 32))
    if "global_batch_size" in config:
        if config["global_batch_size"] % world:
            raise ValueError(f"global_batch_size {config['global_batch_size']} is not a multiple of {world} ranks")
        batch_size = config["global_batch_size"] // world
    train_set = Dataset(train_dir, config)
    if ddp:
        sampler = ShardSampler(train_set, world, rank, shuffle=True, seed=seed, drop_last=True)
        # crop offsets come from the workers' Python RNG, seeded from this
        # generator: per-rank streams, and the global generator is not consumed
        train_loader = DataLoader(train_set, num_workers=num_jobs, sampler=sampler, batch_size=batch_size,
                                  pin_memory=True, drop_last=True, collate_fn=collate_fn,
                                  generator=torch.Generator().manual_seed(seed + 1000003 * (rank + 1)))
    else:
        sampler = None
        train_loader = DataLoader(train_set, num_workers=num_jobs, shuffle=True, batch_size=batch_size,
                                  pin_memory=True, drop_last=True, collate_fn=collate_fn)
    if len(train_loader) == 0:
        raise ValueError(f"{len(train_set)} utterances give no full batch of {batch_size} per rank on {world} rank(s)")

    valid_loader, valid_set = None, []
    if valid_dir is not None and rank == 0:  # rank 0 validates (bin/train.py:79-91)
        try:
            vbs = config.get("valid_batch_size", config.get("batch_size", 1))
            valid_set = Dataset(valid_dir, config, valid=True)
            valid_loader = DataLoader(valid_set, num_workers=num_jobs, shuffle=False, batch_size=vbs,
                                      pin_memory=True, drop_last=False, collate_fn=collate_fn)
        except Exception as e:  # the reference's bare except disables validation silently
            logging.getLogger("logger").warning("validation disabled: %r", e)
            valid_set, valid_loader = [], None

    output_dir = Path(output_dir)
    if rank == 0:
        output_dir.mkdir(parents=True, exist_ok=True)
    if ddp:
        dist.barrier()
    logger = _logger(output_dir, rank)

    logger.info(trainer.get_model_info())
    logger.info("Output directory: {}".format(output_dir))
    logger.info("Training utterances: {}".format(len(train_set)))
    logger.info("Validation utterances: {}".format(len(valid_set)))
    if ddp:
        logger.info("Data parallel: {} ranks ({}), {} utterances per rank per epoch, batch {} per rank".format(
            world, backend, len(sampler), batch_size))
    logger.info("Start traininig...")

    train_log = dict()
    best_loss = {check_loss_kind: np.inf}
    best_iter = 0
    epoch = 0
    while iteration <= max_iter:
        if sampler is not None:
            sampler.set_epoch(epoch)
        epoch += 1
        for i, batch in enumerate(train_loader):
            iteration, loss_detail = trainer.train_step(batch, iteration=iteration)

            for key, val in loss_detail.items():
                train_log.setdefault(key, []).append(val)

            if iteration % iters_per_log == 0 and len(train_log.keys()) > 0:
                means = _ranks_mean(train_log, backend) if ddp else {k: np.mean(v) for k, v in train_log.items()}
                mseg = "Iter {}:".format(iteration)
                for key in train_log:
                    mseg += "  {}: {:.6f}".format(key, means[key])
                logger.info(mseg)
                train_log = dict()

            if iteration % iters_per_checkpoint == 0:
                checkpoint_path = output_dir / "iter.{}".format(iteration)
                if rank == 0:
                    trainer.save_checkpoint(checkpoint_path)
                    logger.info("Saved state dict. to {}".format(checkpoint_path))

            if iteration % iters_per_checkpoint == 0 and valid_loader is not None:
                loss_detail = trainer.valid(valid_loader)
                best_check_loss = np.mean(best_loss[check_loss_kind])
                check_loss = np.mean(loss_detail[check_loss_kind])
                if best_check_loss >= check_loss:
                    best_loss = loss_detail
                    best_iter = iteration
                mseg = "Valid {}:".format(iteration)
                for key, val in loss_detail.items():
                    mseg += "  {}: {:.6f}".format(key, np.mean(val))
                mseg += "  |  Best {}:  {}: {:.6f}".format(best_iter, check_loss_kind, best_check_loss)
                logger.info(mseg)

            if ddp and iteration % iters_per_checkpoint == 0:
                dist.barrier()  # the checkpoint is on disk before any rank moves on

            if iteration > max_iter:
                break

    if rank == 0:
        mseg = "Best model: iteration: {}".format(best_iter)
        for key, val in best_loss.items():
            mseg += "  {}: {:.6f}".format(key, np.mean(val))
        logger.info(mseg)
        best = output_dir / "iter.{}".format(best_iter)
        if best_iter > 0 and best.exists():
            copyfile(str(best), str(output_dir / "model.loss.best"))
        else:
            logger.info("No validated checkpoint: model.loss.best not written")
    logger.info("Finished")
    if ddp:
        dist.barrier()
    return trainer


def main(argv=None):
    import argparse
    parser = argparse.ArgumentParser()
    parser.add_argument("-c", "--config", type=str, default="conf/utt2spks.yaml", help="YAML file for configuration")
    parser.add_argument("--output_dir", type=str, default=None, help="Directory for checkpoint output")
    parser.add_argument("--checkpoint", type=str, default=None, help="checkpoint path to keep training")
    parser.add_argument("--train_dir", type=str, default=None, help="Traininig data dir.")
    parser.add_argument("--valid_dir", type=str, default=None, help="Validation data dir.")
    parser.add_argument("-g", "--gpu", type=str, default="0", help="Using gpu # (single-process runs)")
    parser.add_argument("--backend", type=str, default=None, choices=[None, "nccl", "gloo"],
                        help="data-parallel backend (default: nccl with GPUs, else gloo)")
    args = parser.parse_args(argv)
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        os.environ["CUDA_VISIBLE_DEVICES"] = args.gpu  # bin/train.py:198; under torchrun LOCAL_RANK selects
    try:
        train(args)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
