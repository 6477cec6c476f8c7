"""The data-parallel training entry (vae_npvc_amd/bin/train.py) on the CPU:
ShardSampler gives disjoint per-rank shares whose union is the epoch, every
rank runs the same iterations, rank 0 alone checkpoints, validates and logs,
and the logged means are averaged over the ranks (world size 2, gloo; SURVEY
§8e "Partitioning", ref vae_npvc/bin/train.py:44-76,123-175)."""
import os
import socket
import types

import pytest
import torch
import torch.multiprocessing as mp
import yaml

from vae_npvc_amd.dataset.sampler import ShardSampler


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,world", [(24, 2), (25, 2), (17, 3), (5, 8), (64, 8)])
def test_shard_sampler_disjoint_union_equal_counts(n, world):
    data = list(range(n))
    for epoch in range(3):
        shards = []
        for r in range(world):
            s = ShardSampler(data, world, r, shuffle=True, seed=777, drop_last=True)
            s.set_epoch(epoch)
            shards.append(list(s))
            assert len(shards[-1]) == len(s) == n // world
        flat = [i for sh in shards for i in sh]
        assert len(set(flat)) == len(flat)                        # disjoint
        assert set(flat) <= set(data) and len(flat) == world * (n // world)
        order = ShardSampler(data, world, 0, seed=777).epoch_order() if epoch == 0 else None
        if order is not None:
            assert set(flat) == set(order.tolist())               # the union is the (cut) epoch
    a, b = ShardSampler(data, world, 0, seed=777), ShardSampler(data, world, 0, seed=777)
    b.set_epoch(1)
    if n >= 8:
        assert list(a.epoch_order()) != list(b.epoch_order())     # a new permutation per epoch


def test_shard_sampler_eval_pads_and_leaves_global_rng_alone():
    data = list(range(10))
    g0 = torch.get_rng_state()
    shards = [list(ShardSampler(data, 4, r, shuffle=False, drop_last=False)) for r in range(4)]
    assert torch.equal(torch.get_rng_state(), g0)                  # private generator only
    assert [len(s) for s in shards] == [3, 3, 3, 3]
    assert set(i for s in shards for i in s) == set(data)


def _worker(rank, world, port, cfg_path, out_dir, q):
    try:
        os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank),
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.set_num_threads(1)
        from vae_npvc_amd.bin import train as entry
        args = types.SimpleNamespace(config=cfg_path, output_dir=out_dir, checkpoint=None, train_dir="unused",
                                     valid_dir="unused", backend="gloo")
        tr = entry.train(args)
        import torch.distributed as dist
        dist.destroy_process_group()
        q.put((rank, tr.seen, tr.saved, tr.valids, None))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, None, None, None, traceback.format_exc() + repr(e)))


def _run(tmp_path, world, n_utts, bs, max_iter, per_log, per_ckpt):
    cfg = dict(trainer_type="tests.ddp_stubs:Trainer", dataset_type="tests.ddp_stubs:Utts", n_utts=n_utts,
               n_valid=5, batch_size=bs, max_iter=max_iter, iters_per_log=per_log, iters_per_checkpoint=per_ckpt,
               num_jobs=0, seed=777)
    cfg_path = str(tmp_path / "conf.yaml")
    yaml.safe_dump(cfg, open(cfg_path, "w"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, cfg_path, str(tmp_path / "exp"), q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=180) for _ in ps), key=lambda t: t[0])
    for p in ps:
        p.join(30)
    for r in res:
        assert r[4] is None, r[4]
    return res


def test_train_entry_two_ranks_shard_and_agree(tmp_path):
    n, bs, world = 24, 3, 2
    res = _run(tmp_path, world, n, bs, max_iter=10, per_log=2, per_ckpt=4)
    seen = [r[1] for r in res]
    # same iterations on every rank; like the reference the loop stops after the first step past max_iter
    its = [[it for it, _ in s] for s in seen]
    assert its[0] == its[1] == list(range(1, 12))
    per_epoch = n // (world * bs)  # 4 iterations per epoch
    for e in range(2):             # two whole epochs: disjoint shards covering every utterance
        ids = [[i for it, b in s[e * per_epoch:(e + 1) * per_epoch] for i in b] for s in seen]
        assert not set(ids[0]) & set(ids[1])
        assert sorted(ids[0] + ids[1]) == list(range(n))
    e0 = [i for _, b in seen[0][:per_epoch] for i in b]
    e1 = [i for _, b in seen[0][per_epoch:2 * per_epoch] for i in b]
    assert e0 != e1                # set_epoch: a new permutation each pass
    # rank 0 alone checkpoints and validates
    assert [os.path.basename(p) for p in res[0][2]] == ["iter.4", "iter.8"] and res[1][2] == []
    assert res[0][3] == 2 and res[1][3] == 0
    exp = tmp_path / "exp"
    assert torch.load(exp / "iter.8", weights_only=True) == {"iteration": 8, "rank": 0}
    assert (exp / "model.loss.best").exists()
    log = (exp / "train.log").read_text()
    lines = [l for l in log.splitlines() if " Iter " in l]
    assert [l.split("Iter ")[1].split(":")[0] for l in lines] == ["2", "4", "6", "8", "10"]
    assert all("X like: 1.500000" in l and "Total: 15.000000" in l for l in lines)  # mean over the ranks


def test_train_entry_ragged_epoch_three_ranks(tmp_path):
    n, bs, world = 20, 2, 3   # 6 utterances per rank (2 dropped), 3 batches per epoch
    res = _run(tmp_path, world, n, bs, max_iter=5, per_log=100, per_ckpt=100)
    seen = [r[1] for r in res]
    assert all([it for it, _ in s] == list(range(1, 7)) for s in seen)
    ids = [[i for it, b in s[:3] for i in b] for s in seen]
    flat = [i for x in ids for i in x]
    assert len(flat) == len(set(flat)) == 18
    assert not (tmp_path / "exp" / "model.loss.best").exists()  # nothing validated: no copy (reference crashes)
