"""Data parallelism through the real engine on the GPU: two ranks (gloo
process group, both on cuda:0 — the box has one GPU; RCCL refuses two ranks
on one device) each train on half of the global batch with the HIP kernels,
and must reproduce the single-process step on the whole batch (SURVEY §8e:
gradient mean all-reduce, EMA-statistics sum all-reduce, dead-code rows
assembled from the owning ranks, broadcast of the initial weights).  The
CPU test tests/test_ddp_gloo.py checks the same algorithm on the oracle; this
one runs the engine's own distributed code (engine/step.py, parallel/ddp.py).
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD, B, T, STEPS = 2, 4, 128, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batches(y_num):
    g = torch.Generator().manual_seed(2024)
    return [(torch.randn(B, 80, T, generator=g), torch.randint(0, y_num, (B, 1), generator=g)) for _ in range(STEPS)]


def _run(rank, world, port, dtype, q):
    """One training process: rank `rank` of `world` (world 1 = the reference)."""
    try:
        import torch.distributed as dist
        from tests.helpers import cfg_of, make_trainer
        torch.cuda.set_device(0)
        if world > 1:
            dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        cfg = cfg_of("vcc20", compute_dtype=dtype)
        np.random.seed(11)
        tr = make_trainer(cfg, 3)
        torch.manual_seed(11)  # the same CPU generator on every rank: shared randperm of the global batch
        per = B // world
        losses = []
        for x, y in _batches(cfg["y_num"]):
            sl = slice(rank * per, (rank + 1) * per)
            _, det = tr.train_step((x[sl].cuda(), y[sl].cuda()))
            losses.append(dict(det))
        torch.cuda.synchronize()
        flat = tr.engine.flat_p.detach().cpu().numpy()
        # a digest of all 31.3M weights (rank equality) and every 16th weight (numerics)
        q.put((rank, world, (hashlib.sha1(flat.tobytes()).hexdigest(), flat[::16].copy()),
               tr.model.quantizer.embeddings.detach().cpu().numpy(), losses))
        if world > 1:
            dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, world, None, None, repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-5), ("bf16", 2e-3)])
def test_two_rank_engine_step_equals_global_batch_step(dtype, tol):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_keep = {k: os.environ.get(k) for k in ("MASTER_ADDR",)}
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    try:
        ps = [ctx.Process(target=_run, args=(r, WORLD, port, dtype, q)) for r in range(WORLD)]
        ps.append(ctx.Process(target=_run, args=(0, 1, 0, dtype, q)))  # single-process reference, whole batch
        for p in ps:
            p.start()
        res = [q.get(timeout=240) for _ in ps]
        for p in ps:
            p.join(60)
    finally:
        if env_keep["MASTER_ADDR"] is None:
            os.environ.pop("MASTER_ADDR", None)
    for r in res:
        assert r[2] is not None, r[4]
    ref = next(r for r in res if r[1] == 1)
    ranks = sorted((r for r in res if r[1] == WORLD), key=lambda r: r[0])
    # every rank holds the same weights and codebook
    assert ranks[0][2][0] == ranks[1][2][0]
    assert np.array_equal(ranks[0][3], ranks[1][3])
    # ... and they are the global-batch step's (fp32; EMA scatter atomics reorder sums)
    d = np.linalg.norm(ranks[0][2][1] - ref[2][1]) / np.linalg.norm(ref[2][1])
    assert d < tol, d
    dE = np.linalg.norm(ranks[0][3] - ref[3]) / np.linalg.norm(ref[3])
    assert dE < 10 * tol, dE
    # the mean of the per-rank reconstruction losses is the global one
    for s in range(STEPS):
        mean_x = np.mean([r[4][s]["X like"] for r in ranks])
        assert abs(mean_x - ref[4][s]["X like"]) <= 10 * tol * abs(ref[4][s]["X like"])
