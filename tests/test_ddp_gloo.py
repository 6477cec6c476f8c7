"""Data parallelism at world_size 2 on the CPU (gloo): the engine's Comm
(bucketed async mean all-reduce, sum all-reduce) and the SURVEY §8e parity
target — two ranks, each training on half of the global batch with the
gradient mean all-reduce, the EMA-statistics sum all-reduce and the
owned-rows assembly of the dead-code rows, reproduce the single-process step
on the whole batch (the oracle restatement on both sides)."""
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.helpers import cfg_of

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, port):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    torch.set_num_threads(2)


def small_cfg():
    cfg = cfg_of("vcc20")
    cfg = copy.deepcopy(cfg)
    cfg["encoder"]["out_channels"] = [64]
    cfg["encoder"]["stacks"] = [2]
    cfg["decoder"]["out_channels"] = [64]
    cfg["decoder"]["stacks"] = [2]
    cfg["decoder"]["skip_channels"] = 32
    cfg["decoder"]["cond_channels"] = 16
    cfg["y_dim"] = 16
    cfg["z_num"] = 64
    return cfg


# ---------------------------------------------------------------- Comm
def _comm_worker(rank, port, q):
    try:
        _init(rank, port)
        from vae_npvc_amd.parallel.ddp import Comm
        comm = Comm(bucket_bytes=64 * 4)  # 64 floats per bucket: many buckets
        flat = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        comm.grads_ready(flat, 0, 600)
        comm.grads_ready(flat, 600, 1000)
        comm.finish()
        want = torch.arange(1000, dtype=torch.float32) * 1.5  # mean of x1 and x2
        s = torch.full((3,), float(rank + 1))
        work = comm.all_reduce_sum(s, async_op=True)
        comm.wait(work, "ema")
        m = comm.mean_scalars(torch.tensor([float(rank)]))
        # diagnostics (bench.py "comm"): 1000 gradient floats in 64-float buckets
        # (10 + 7) plus the 3-float sum; waits are timed under RCCL only
        nbytes, calls, grad_ms, ema_ms = comm.stats()
        ok_stats = (nbytes, calls, grad_ms, ema_ms) == (1003 * 4, 18, 0, 0)
        comm.reset_stats()
        ok_stats = ok_stats and comm.stats() == (0, 0, 0, 0)
        # grad_sync "end": runs held until finish(), adjacent ones merged (here out of
        # order: 600-1000 then 0-600 -> one 1000-float run = 16 buckets), same values
        late = Comm(bucket_bytes=64 * 4, overlap=False)
        flat2 = torch.arange(1000, dtype=torch.float32) * (rank + 1)
        late.grads_ready(flat2, 600, 1000)
        late.grads_ready(flat2, 0, 600)
        ok_late = late.stats()[1] == 0 and torch.equal(flat2, torch.arange(1000, dtype=torch.float32) * (rank + 1))
        late.finish()
        ok_late = ok_late and torch.equal(flat2, want) and late.stats()[:2] == (1000 * 4, 16) and not late.held
        q.put((rank, torch.equal(flat, want) and ok_stats and ok_late, s.tolist(), m.item()))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None, None))


def test_comm_bucketed_mean_and_sum():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_comm_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    for rank, ok, s, m in res:
        assert ok is True, ok
        assert s == [3.0, 3.0, 3.0]
        assert m == 0.5


# ---------------------------------------------------------------- step parity
def _ddp_step_worker(rank, port, cfg, B, T, steps, q):
    try:
        _init(rank, port)
        from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict
        from vae_npvc_amd.parallel.ddp import Comm, owned_rows
        torch.manual_seed(11)  # identical CPU generator on every rank (shared randperm)
        np.random.seed(11)
        tr = OracleTrainer(cfg, seeded_state_dict(cfg, 1))
        comm = Comm(bucket_bytes=1 << 16)
        model = tr.model
        n_local = (B // WORLD) * T

        def reduce_sum(t):
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            return t

        def pick_rows(z):
            if z.shape[0] * WORLD < model.K:
                # N_global < K: every rank tiles the gathered global batch with the
                # same CPU generator, so all ranks draw identical rows (no SUM)
                parts = [torch.empty_like(z) for _ in range(WORLD)]
                dist.all_gather(parts, z.contiguous())
                zt = model._tile(torch.cat(parts))
                return zt[torch.randperm(zt.shape[0])][: model.K]
            # every rank draws randperm(N_global); owners fill, SUM assembles
            perm = torch.randperm(z.shape[0] * WORLD)[: model.K]
            loc = owned_rows(perm, rank * n_local, n_local)
            out = torch.zeros(model.K, z.shape[1])
            mine = loc >= 0
            out[mine] = z[loc[mine]]
            return reduce_sum(out)

        def grad_hook(params):
            flat = torch.cat([p.grad.reshape(-1) for p in params])
            comm.grads_ready(flat, 0, flat.numel())
            comm.finish()
            off = 0
            for p in params:
                p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
                off += p.numel()

        model.reduce_sum, model.pick_rows, tr.grad_hook = reduce_sum, pick_rows, grad_hook
        x, y = seeded_batch(cfg, B, T, 5)
        sl = slice(rank * (B // WORLD), (rank + 1) * (B // WORLD))
        losses = []
        for _ in range(steps):
            _, det = tr.train_step((x[sl], y[sl]))
            losses.append((det["X like"], det["VQ loss"]))
        # numpy copies: pickled by value (tensors would travel as shared-memory handles
        # that vanish when this process exits)
        st = {k: v.detach().numpy().copy() for k, v in model.params.items()}
        q.put((rank, losses, st, model.embeddings.numpy().copy(), model.emb_elem.numpy().copy()))
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc() + repr(e), None, None, None))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("B,T", [(4, 64), (2, 16)])  # (2, 16): N_global = 32 < K = 64, the _tile path
def test_two_rank_step_equals_global_batch_step(B, T):
    from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict
    cfg, steps = small_cfg(), 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_step_worker, args=(r, port, cfg, B, T, steps, q)) for r in range(WORLD)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=500) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(30)
    for r in res:
        assert r[2] is not None, r[1]

    torch.manual_seed(11)
    np.random.seed(11)
    ref = OracleTrainer(cfg, seeded_state_dict(cfg, 1))
    x, y = seeded_batch(cfg, B, T, 5)
    ref_losses = []
    for _ in range(steps):
        _, det = ref.train_step((x, y))
        ref_losses.append((det["X like"], det["VQ loss"]))

    # N_global < K: each frame sits between its own noisy tiled copies at squared
    # distances ~1e-4 against |z|^2 ~ 1e2, so the argmin between them flips with
    # the matmul blocking of the local vs global batch (fp32 rounding ~1e-5):
    # the commitment loss is then only reproducible to ~1%, and the flips change
    # which codes survive the first EMA update: later steps are compared only
    # between the ranks (which must agree exactly: the rows are drawn from the
    # gathered global batch, not from each rank's own frames)
    tiled = B * T < cfg["z_num"]
    for s in range(1 if tiled else steps):
        # frame_mean losses: the global value is the mean over the equal shards
        for j in range(2):
            got = 0.5 * (res[0][1][s][j] + res[1][1][s][j])
            rt = 2e-2 if (tiled and j == 1) else 2e-5
            assert got == pytest.approx(ref_losses[s][j], rel=rt), (s, j, res[0][1], res[1][1], ref_losses)
    # both ranks hold identical weights and codebooks
    for k in res[0][2]:
        assert np.array_equal(res[0][2][k], res[1][2][k]), k
    assert np.array_equal(res[0][3], res[1][3])
    if tiled:
        return
    # ... equal to the single-process global-batch step (fp32 summation order differs)
    for k, v in ref.model.params.items():
        v = v.detach().numpy()
        d = np.linalg.norm(res[0][2][k] - v) / max(np.linalg.norm(v), 1e-12)
        assert d < 1e-4, (k, d)
    assert np.allclose(res[0][3], ref.model.embeddings.numpy(), rtol=1e-4, atol=1e-6)
    assert np.allclose(res[0][4], ref.model.emb_elem.numpy(), rtol=1e-6)
