"""The RCCL branch of the data-parallel code on the GPU (backend "nccl" = RCCL
on ROCm), in a world-size-1 process group: the box has one GPU and RCCL
refuses two ranks on one device, so this is the only way to execute the
device-tensor collectives before the driver's 8-GPU run.

  * Comm.grads_ready / finish: bucketed async ReduceOp.AVG all-reduces of a
    device buffer written by work queued on the compute stream behind a long
    sleep kernel, read back by work queued after finish() -- values exact
    (the stream ordering RCCL's internal stream must respect both ways);
  * Comm.all_gather_cat / mean_scalars / all_reduce_sum(async) on device tensors;
  * the engine with the communicator attached (every collective of the step:
    initial broadcast, per-group gradient all-reduces, the EMA-statistics
    bundle, owned-rows assembly) equals the plain engine bit for bit over
    three steps, and every gradient is reduced exactly once per step -- with
    the weight-norm backward batched every 5 groups (default), per group and
    for all groups at once;
  * bin/train.py's nccl initialisation path from torchrun-style env
    (setup_distributed), world size 1.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _sha(t):
    return hashlib.sha1(t.detach().cpu().numpy().tobytes()).hexdigest()


def _worker(port, q):
    try:
        os.environ.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        from vae_npvc_amd.bin.train import setup_distributed
        from vae_npvc_amd.parallel.ddp import Comm
        # bin/train.py's path treats WORLD_SIZE=1 as single-process: initialise explicitly
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        torch.cuda.set_device(dev)
        assert setup_distributed() == (1, 0, None)
        out = {}
        comm = Comm(bucket_bytes=1 << 16)  # 16 K floats per bucket: many buckets
        out["backend"] = comm.backend
        src = torch.randn(200_000, device=dev)
        flat = torch.zeros_like(src)
        torch.cuda._sleep(20_000_000)           # the producer is late ...
        flat.copy_(src).mul_(3.0)               # ... and queued on the compute stream
        comm.grads_ready(flat, 0, 120_000)
        comm.grads_ready(flat, 120_000, 200_000)
        comm.finish()
        flat.add_(1.0)                          # consumer after finish()
        torch.cuda.synchronize()
        out["avg_exact"] = bool(torch.equal(flat, src * 3.0 + 1.0))
        g = comm.all_gather_cat(src[:1000].view(10, 100))
        out["gather_exact"] = bool(g.is_cuda and torch.equal(g, src[:1000].view(10, 100)))
        m = comm.mean_scalars(torch.tensor([2.5, -1.0], device=dev))
        out["mean"] = m.cpu().tolist()
        s = torch.full((7,), 3.0, device=dev)
        torch.cuda._sleep(10_000_000)
        s.mul_(2.0)
        comm.all_reduce_sum(s, async_op=True).wait()
        s.add_(1.0)
        out["sum"] = s.cpu().tolist()

        # the engine's data-parallel step vs the plain step
        from oracle.vqvae_cpu import seeded_batch
        from tests.helpers import cfg_of, load_fixture, make_trainer
        meta, _ = load_fixture("step_vcc20")
        cfg = cfg_of("vcc20", compute_dtype="fp32")
        runs = []
        # plain, all-reduce beside the backward (weight-norm backward batched every 5 groups, every
        # group, all groups at once), all after it
        for ddp, chunk in ((False, 5), (True, 5), ("end", 5), (True, 1), (True, 1000)):
            tr = make_trainer(dict(cfg, engine={"wn_bwd_ddp_groups": chunk}), meta["wseed"])
            eng = tr.engine
            calls = []
            if ddp:
                c2 = Comm(overlap=ddp is True)
                real = c2.grads_ready

                def rec(flat_, lo, hi, _real=real):
                    calls.append((lo, hi))
                    _real(flat_, lo, hi)
                c2.grads_ready = rec
                eng.attach_comm(c2)
                dist.broadcast(eng.flat_p, 0)
            torch.manual_seed(meta["tseed"])
            np.random.seed(meta["nseed"])
            dets, per_step = [], []
            for st in range(meta["steps"]):
                x, y = seeded_batch(cfg, meta["B"], meta["T"], meta["bseed"] + st)
                n0 = len(calls)
                _, det = tr.train_step((x.cuda(), y.cuda()))
                dets.append(dict(det))
                per_step.append(sorted(calls[n0:]))
            torch.cuda.synchronize()
            runs.append(dict(p=_sha(eng.flat_p), e=_sha(tr.model.quantizer.embeddings), d=dets, calls=per_step,
                             n=eng.n_params))
        out["engine"] = runs
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((None, traceback.format_exc() + repr(e)))


def test_rccl_world1_comm_and_engine_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    out, err = q.get(timeout=300)
    p.join(60)
    assert err is None, err
    assert out["backend"] == "nccl"
    assert out["avg_exact"] and out["gather_exact"]
    assert out["mean"] == [2.5, -1.0]
    assert out["sum"] == [7.0] * 7
    plain, ddp, late, per_group, one = out["engine"]
    for d in (ddp, late, per_group, one):
        assert d["p"] == plain["p"] and d["e"] == plain["e"]       # bit-identical weights and codebook
        assert d["d"] == plain["d"]                                # identical loss dicts
        for calls in d["calls"]:                                   # every gradient reduced exactly once per step
            covered = 0
            for (lo, hi), nxt in zip(calls, calls[1:] + [(d["n"], None)]):
                assert lo < hi <= nxt[0]
                covered += hi - lo
            assert covered == d["n"]
    assert len(ddp["calls"][0]) > 3                                # reduced in several runs during the backward
    assert len(per_group["calls"][0]) > len(ddp["calls"][0]) > len(one["calls"][0])
