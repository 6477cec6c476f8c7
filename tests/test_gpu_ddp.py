"""Data parallelism through the real engine on the GPU, against the
reference's own fixture (the parity target of N ranks is the
single-process reference step on the global batch).

Two ranks (gloo process group, both on cuda:0 -- the box has one GPU and RCCL
refuses two ranks on one device) each train on two of the four utterances of
tests/golden/step_vcc20 (the reference's B=4 x T=128, three steps) with the
HIP kernels and the engine's own distributed code (engine/step.py,
parallel/ddp.py): per-group gradient mean all-reduces, the EMA-statistics sum
all-reduce, dead-code rows assembled from the owning ranks, broadcast of the
initial weights.  Checked against the REFERENCE values, not against a HIP
world-1 run:
  * per-rank frame-mean losses average to the reference's global losses;
  * the EMA diagnostics (global statistics) equal the reference's on each rank;
  * the all-reduced step-1 gradients have the reference's norms;
  * the parameters after three steps have the reference's norms;
  * both ranks hold bit-identical weights (SHA-1 of all 31.3M) and codebooks.
A second case runs the N_global < K path (_tile, layers_vq.py:183-190) and
checks that the ranks stay identical.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank, world, port, dtype, prefix, T_override, q, engine=None):
    try:
        import torch.distributed as dist
        from oracle.vqvae_cpu import seeded_batch
        from tests.helpers import cfg_of, load_fixture, make_trainer
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        meta, _ = load_fixture(prefix)
        cfg = cfg_of(meta["config"], compute_dtype=dtype, **({"engine": engine} if engine else {}))
        B, T = meta["B"], T_override or meta["T"]
        tr = make_trainer(cfg, meta["wseed"])
        eng = tr.engine
        assert eng.world == world and eng.rank == rank
        torch.manual_seed(meta["tseed"])  # the same CPU generator on every rank (shared randperm)
        np.random.seed(meta["nseed"])
        per = B // world
        sl = slice(rank * per, (rank + 1) * per)
        losses, grads = [], None
        for s in range(meta["steps"]):
            x, y = seeded_batch(cfg, B, T, meta["bseed"] + s)
            _, det = tr.train_step((x[sl].cuda(), y[sl].cuda()))
            losses.append(dict(det))
            if s == 0:
                grads = {n: float(eng.g(p).double().norm()) for n, p in tr.model.named_parameters()}
        torch.cuda.synchronize()
        flat = eng.flat_p.detach().cpu().numpy()
        params = {n: float(p.detach().double().norm()) for n, p in tr.model.named_parameters()}
        q.put((rank, hashlib.sha1(flat.tobytes()).hexdigest(), tr.model.quantizer.embeddings.detach().cpu().numpy(),
               losses, grads, params))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put((rank, None, None, repr(e) + traceback.format_exc(), None, None))


def _spawn(dtype, prefix, T_override=None, engine=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    keep = os.environ.get("MASTER_ADDR")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    try:
        ps = [ctx.Process(target=_run, args=(r, WORLD, port, dtype, prefix, T_override, q, engine))
              for r in range(WORLD)]
        for p in ps:
            p.start()
        res = [q.get(timeout=240) for _ in ps]
        for p in ps:
            p.join(60)
    finally:
        if keep is None:
            os.environ.pop("MASTER_ADDR", None)
    for r in res:
        assert r[1] is not None, r[3]
    return sorted(res, key=lambda r: r[0])


def _rel(a, b):
    return abs(a - b) / max(abs(b), 1e-12)


@pytest.mark.parametrize("prefix,dtype", [("step_vcc20", "fp32"), ("step_vcc20", "bf16"), ("step_aishell3", "fp32"),
                                          ("step_aishell3", "bf16"), ("step_vcc20_multi", "fp32")])
def test_two_rank_engine_step_matches_reference_golden(prefix, dtype):
    """fp32: losses 1e-4 at step 1 and 1e-3 later, gradient norms 2e-3 (as the
    single-process golden test), parameters after 3 steps 1e-3.  bf16 (the
    bench dtype): losses 1e-2 (VQ loss 2e-2), gradient norms 5e-2, parameters 1e-2.
    aishell3 (BASELINE config 4: 160 mel, K=128, skip 256, jitter 0.12, bf16
    as the config states) needs the same numpy stream on every rank: each
    rank draws the single-process jitter map.  vcc20_multi is the general topology (two stages, stride-2
    resampling, dilation, stack_layers 2, kernel 5)."""
    from tests.helpers import load_fixture
    meta, _ = load_fixture(prefix)
    ranks = _spawn(dtype, prefix)
    assert ranks[0][1] == ranks[1][1]  # identical weights on every rank
    assert np.array_equal(ranks[0][2], ranks[1][2])  # ... and codebooks
    f32 = dtype == "fp32"
    for s in range(meta["steps"]):
        ref = meta["detail"][s]
        lt = (1e-4 if s == 0 else 1e-3) if f32 else 1e-2
        for k in ("X like", "Total"):  # frame means over equal shards: the global value is their mean
            got = np.mean([r[3][s][k] for r in ranks])
            assert _rel(got, ref[k]) <= lt, (s, k, got, ref[k])
        got = np.mean([r[3][s]["VQ loss"] for r in ranks])
        # bf16: the commitment loss follows the codebook assignments, whose near-tie flips
        # amplify rounding differences step by step -- 2e-2 as the other bf16 step tests
        # (test_gpu_configs.py); fp32 keeps lt
        # (3e-2 from step 2 on: after an Adam step the bf16 roundings have moved the codebook
        # assignments of the 512 frames away from the fp32 reference's -- 2.1% measured on
        # aishell3 with jitter at step 3, 0.3-1.2% elsewhere).  The bar does not hide the
        # three-workgroups-per-CU 1x1 kernels that became the default with it: they equal the
        # round-4 kernels (kernel_policy 5) bit for bit over whole steps
        # (test_gpu_step.py::test_three_per_cu_1x1_policy_is_bit_identical)
        vt = lt if f32 else (2e-2 if s == 0 else 3e-2)
        assert abs(got - ref["VQ loss"]) <= vt * abs(ref["VQ loss"]) + 1e-6, (s, got, ref["VQ loss"])
        if s == 0 or f32:  # EMA diagnostics come from the all-reduced statistics: global on every rank
            # bf16: 512 frames over K = 128 codes; one frame whose nearest code flips under the
            # bf16 operand rounding moves the entropy (exp of the code-histogram entropy) by ~0.5%
            dt = max(lt, 1e-4) if f32 else 3e-2
            for k in ("entropy", "used_curr", "usage"):
                for r in ranks:
                    assert _rel(r[3][s][k], ref[k]) <= dt, (s, k, r[3][s][k], ref[k])
    gt = 2e-3 if f32 else 5e-2
    for n, ref in meta["grads"].items():
        for r in ranks:
            assert abs(r[4][n] - ref["norm"]) <= gt * ref["norm"] + 1e-9, (n, r[4][n], ref["norm"])
    pt = 1e-3 if f32 else 1e-2
    for n, ref in meta["params_after"].items():
        assert _rel(ranks[0][5][n], ref["norm"]) <= pt, (n, ranks[0][5][n], ref["norm"])


def test_two_rank_tile_path_keeps_ranks_identical():
    """N_global = 4 x 32 = 128 < K = 512: the dead-code / init rows come from
    tiling the gathered global batch with noise drawn identically on every
    rank (engine _tile_rows), so the ranks' codebooks stay bit-identical."""
    ranks = _spawn("fp32", "step_vcc20", T_override=32)
    assert ranks[0][1] == ranks[1][1]
    assert np.array_equal(ranks[0][2], ranks[1][2])
    for s in range(3):  # the EMA diagnostics are global statistics
        for k in ("entropy", "used_curr", "usage", "diff_emb"):
            assert ranks[0][3][s][k] == ranks[1][3][s][k], (s, k)


@pytest.mark.timeout(600)
def test_bench_two_ranks_reports_comm_block():
    """bench.py's N > 1 path end to end on the box's one GPU: --gpus 2 launches
    two ranks under torch.distributed.run (here with the gloo process group,
    since RCCL refuses two ranks on one device), times the barrier-bracketed
    steps as the max over ranks and prints the line with the `comm` block
    (bytes all-reduced and collectives per step, per-rank waits, grad_sync),
    for the all-reduce beside the backward and after it."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lines = {}
    for mode in ("overlap", "end"):
        cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
               "--dist-backend", "gloo", "--grad-sync", mode, "--no-cpu-baseline", "--fp32-steps", "0",
               "--vq-reps", "0", "--no-probe"]
        env = dict(os.environ)
        env.pop("WORLD_SIZE", None)
        r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=500)
        assert r.returncode == 0, r.stderr[-3000:]
        js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(js) == 1, r.stdout[-2000:]
        lines[mode] = json.loads(js[0])
    for mode, d in lines.items():
        assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0, d
        c = d["comm"]
        assert c["backend"] == "gloo" and c["grad_sync"] == mode, c
        # every fp32 gradient once per step (31.3 M params) plus the EMA statistics bundle
        assert 31_000_000 * 4 < c["bytes_per_step"] < 32_000_000 * 4 + (8 << 20), c
        assert len(c["grad_wait_ms"]) == 2 and len(c["ema_wait_ms"]) == 2, c
    assert lines["end"]["comm"]["bytes_per_step"] == lines["overlap"]["comm"]["bytes_per_step"]
    assert lines["end"]["comm"]["collectives_per_step"] <= lines["overlap"]["comm"]["collectives_per_step"]


@pytest.mark.parametrize("prefix,dtype", [("step_vcc20", "bf16"), ("step_aishell3", "fp32")])
def test_two_rank_two_stream_backward_is_bit_identical(prefix, dtype):
    """EngineOptions.bwd_streams under data parallel (round 6): the encoder
    backward on the second stream from the VQ forward on, its gradient runs
    all-reduced from that stream (_wn_enc_run).  The weights after three steps
    (SHA-1 of all 31.3M), the codebooks and every loss equal the one-stream
    schedule's bit for bit on both ranks: the all-reduces sum the same
    elements in the same rank order, whatever their bucketing."""
    a = _spawn(dtype, prefix)
    b = _spawn(dtype, prefix, engine={"bwd_streams": False})
    for ra, rb in zip(a, b):
        assert ra[1] == rb[1], ra[0]
        assert np.array_equal(ra[2], rb[2])
        assert ra[3] == rb[3]
