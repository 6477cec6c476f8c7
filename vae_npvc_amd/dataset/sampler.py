"""Utterance sharding for data-parallel training (SURVEY §8e "Partitioning").

The reference trains on one GPU with `DataLoader(shuffle=True, drop_last=True)`
(vae_npvc/bin/train.py:67-76): every epoch is a fresh permutation of the
utterances drawn from the global torch generator, cut into batches.  With one
process per GPU, a plain shuffled loader on every rank would draw the SAME
permutation on every rank (bin/train.py:44-46 seeds the global generators
identically, and data parallelism needs them identical for the EMA codebook's
shared randperm), so every rank would train on the same batches.

`ShardSampler` gives each rank a disjoint share of one epoch permutation:

* the permutation of epoch e is `torch.randperm(n)` on a private generator
  seeded with `seed + e` -- identical on every rank, and it never touches the
  global generators, whose stream stays identical across ranks;
* drop_last (training): the permutation is cut to `world * (n // world)`
  utterances, rank r takes positions r, r + world, r + 2*world, ...; the
  shards are disjoint and their union is the cut epoch, and every rank holds
  the same count, so every rank's loader yields the same number of batches
  and the gradient all-reduces of a step always pair up;
* without drop_last (evaluation), the permutation is padded by wrapping to a
  multiple of `world` (each utterance at least once, a few twice).

`set_epoch(e)` selects the permutation; the training entry calls it at the top
of every pass over the loader (vae_npvc_amd/bin/train.py).
"""
import math

import torch


class ShardSampler(torch.utils.data.Sampler):
    def __init__(self, dataset, num_replicas, rank, shuffle=True, seed=0, drop_last=True):
        if num_replicas < 1 or not 0 <= rank < num_replicas:
            raise ValueError(f"ShardSampler: rank {rank} outside [0, {num_replicas})")
        self.n = len(dataset)
        self.world, self.rank = int(num_replicas), int(rank)
        self.shuffle, self.seed, self.drop_last = bool(shuffle), int(seed), bool(drop_last)
        self.epoch = 0
        if drop_last:
            self.per_rank = self.n // self.world
        else:
            self.per_rank = math.ceil(self.n / self.world)
        self.total = self.per_rank * self.world

    def set_epoch(self, epoch):
        self.epoch = int(epoch)

    def epoch_order(self):
        """The whole epoch's utterance order (identical on every rank)."""
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g)
        else:
            order = torch.arange(self.n)
        if self.drop_last:
            return order[: self.total]
        if self.total > self.n:  # pad by wrapping (n >= 1)
            reps = math.ceil((self.total - self.n) / max(1, self.n))
            order = torch.cat([order] + [order] * reps)[: self.total]
        return order

    def __iter__(self):
        return iter(self.epoch_order()[self.rank: self.total: self.world].tolist())

    def __len__(self):
        return self.per_rank
