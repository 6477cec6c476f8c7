#!/usr/bin/env python3
"""Benchmark of the VQ-VAE training step (BASELINE.json metric): mel-frames/s
of one full Trainer.train_step (forward, backward, grad all-reduce, clip,
Adam, StepLR, EMA codebook) on synthetic 80-dim mel batches.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]

N > 1: one rank per GPU (RCCL over xGMI); each rank trains 64 x 256 frames
(weak scaling, global batch 64*N).  Under torch.distributed.run (WORLD_SIZE
set) this process is one rank; started directly with --gpus N > 1 it
launches torch.distributed.run itself as a child process (the parent never
touches the GPU) and exits with its status.
Rank 0 prints ONE JSON line.  Workload = BASELINE configs[1] (vcc20 VQ-VAE,
codebook 512, 80 mel, batch 64 x 256 frames per GPU, bf16 conv GEMMs with
fp32 accumulation; statistics, VQ and optimizer in fp32).  Weights are random
(seeded), data synthetic N(0,1) mel + uniform speaker ids: no network.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import yaml  # noqa: E402

B_PER_GPU, T_FRAMES = 64, 256
FLOP_PER_FRAME = 178.9e6        # algorithmic conv GEMM + VQ distance FLOPs per mel-frame
PEAK_BF16 = 2.5e15              # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32 = 157.3e12
HBM_PEAK = 8.0e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--config", default="vcc20", choices=["vcc20", "aishell3"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--fp32-steps", type=int, default=5,
                    help="N=1: also time this many fp32 (parity-mode) steps, reported under 'fp32' (0 = skip)")
    ap.add_argument("--vq-reps", type=int, default=50, help="VQ kernel launches timed for the 'vq' roofline")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-launch GEMM event probe "
                    "(default: the dominant kernel's launches in every --probe-every-th timed step; "
                    "VQX_BENCH_KERNELS=1/2: every GEMM launch of those steps, per kernel / per layer)")
    ap.add_argument("--probe-every", type=int, default=10,
                    help="probe one step in this many of the timed region (each stamped launch idles the "
                         "stream ~6.5 us: 10 launches in one step of ten cost 0.1%% of the step)")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="run the step on a stream that leaves this many CUs idle (vqx_stream_create_cu_mask): "
                         "the cost of co-resident work such as RCCL's all-reduce kernels")
    ap.add_argument("--grad-sync", default="overlap", choices=["overlap", "end"],
                    help="N>1: gradient all-reduces beside the backward (default) or all after it")
    ap.add_argument("--no-read-loss", dest="read_loss", action="store_false",
                    help="skip the second timed loop that reads loss_detail every step (ms_per_step_read_loss)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 process group (nccl = RCCL; gloo lets tests run several ranks on one GPU)")
    return ap.parse_args()


def cpu_baseline(cfg, steps):
    """The CPU oracle (torch-CPU fp32 restatement of the reference step, validated
    against the reference's golden vectors) on this host's cores, same workload."""
    from oracle.vqvae_cpu import OracleTrainer, seeded_batch, seeded_state_dict
    threads = os.cpu_count() or 1
    threads = min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)))
    torch.set_num_threads(threads)
    ocfg = dict(cfg)
    tr = OracleTrainer(ocfg, seeded_state_dict(ocfg, 1))
    x, y = seeded_batch(ocfg, B_PER_GPU, T_FRAMES, 0)
    tr.train_step((x, y))  # warm-up (includes EMA init)
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.train_step((x, y))
    dt = (time.perf_counter() - t0) / steps
    return {"value": B_PER_GPU * T_FRAMES / dt, "unit": "mel-frames/s", "cores": threads, "kind": "port",
            "sample": f"{steps} timed steps (+1 warm-up) of the oracle train step at B={B_PER_GPU}x{T_FRAMES}, fp32, "
                      f"torch-CPU {torch.__version__}, s/step={dt:.2f}"}


def launch_ranks(n):
    """--gpus N > 1 without a launcher: run N ranks under torch.distributed.run
    (127.0.0.1 rendezvous) as a child process; the parent never initialises
    the GPU (no exec from a GPU-initialised process)."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def time_vq(tr, reps):
    """The VQ distance kernel (distance, argmin, gather, commitment partials +
    their ordered sum; vqx_vq_forward without statistics) re-launched `reps`
    times on the step's own workspace (N = 16,384 frames, K codes, D = 128),
    timed with events on the stream it runs on; `us_with_stats` adds the EMA
    statistics (sort + segmented sums) as the step runs them.  Algorithmic
    bytes: z (N*D f32) + E (K*D f32) + idx (N int64) = 536 B/frame + E
    (SURVEY §8d); FLOPs 2*N*K*D."""
    from vae_npvc_amd import ops
    eng = tr.engine
    w = eng._ws[(B_PER_GPU, T_FRAMES, True)]
    q = tr.model.quantizer
    N, D, K = w.Nz, eng.dims["Z"], eng.dims["K"]
    base = (w.z, q.embeddings, w.idx, w.zq, w.zq_c, w.stats[1:2], w.vq_part)

    def timed(args):
        for _ in range(3):
            ops.vq_forward(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ops.vq_forward(*args)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / reps
    t = timed(base)
    t_stats = timed(base + (w.bsum, w.bcnt))
    nbytes = N * D * 4 + K * D * 4 + N * 8
    flops = 2.0 * N * K * D
    return {"kernel": "vqx::vq_forward_kernel", "us": round(t * 1e6, 2), "us_with_stats": round(t_stats * 1e6, 2),
            "bytes": nbytes, "flops": flops,
            "hbm_GBps": round(nbytes / t / 1e9, 1), "hbm_frac": round(nbytes / t / HBM_PEAK, 4),
            "tflops": round(flops / t / 1e12, 2), "mfma_f32_frac": round(flops / t / PEAK_F32, 4),
            "roofline_frac": round(max(nbytes / HBM_PEAK, flops / PEAK_F32) / t, 4),
            "bound": "mfma_f32" if flops / PEAK_F32 > nbytes / HBM_PEAK else "hbm", "launches": reps}


def time_fp32(cfg, steps, dev):
    """The same workload in the parity dtype (fp32 GEMMs on v_mfma_f32_32x32x2_f32):
    `steps` timed train steps after 2 warm-up steps, 1 GPU."""
    from vae_npvc_amd.trainer.basic import Trainer
    c = dict(cfg, compute_dtype="fp32")
    tr = Trainer(c)
    mel = c["encoder"]["in_channels"][0]
    gen = torch.Generator(device="cpu").manual_seed(4321)
    x = torch.randn(B_PER_GPU, mel, T_FRAMES, generator=gen).to(dev)
    y = torch.randint(0, c["y_num"], (B_PER_GPU, 1), generator=gen).to(dev)
    for _ in range(2):
        _, det = tr.train_step((x, y))
    dict(det)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.train_step((x, y))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    flops = FLOP_PER_FRAME * B_PER_GPU * T_FRAMES
    return {"value": round(B_PER_GPU * T_FRAMES / dt, 1), "unit": "mel-frames/s", "ms_per_step": round(1e3 * dt, 3),
            "steps": steps, "dtype": "fp32", "step_mfma_frac": round(flops / dt / PEAK_F32, 4)}


def time_read_loss(tr, xs, ys, steps, world):
    """ms per step of the timed loop with the step's loss dict read on the host
    after every step, as the reference's training loop does
    (/root/reference/vae_npvc/bin/train.py:128-132: train_log[key].append(val)
    for every key, every iteration); max over ranks."""
    n = len(xs)
    for i in range(2):
        dict(tr.train_step((xs[i % n], ys[i % n]))[1])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    log = {}
    t0 = time.perf_counter()
    for i in range(steps):
        _, det = tr.train_step((xs[i % n], ys[i % n]))
        for k, v in det.items():
            log.setdefault(k, []).append(v)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    return 1e3 * el / steps


def committed_traffic(symbol):
    """HBM bytes per launch of `symbol` from the newest committed PMC summary
    (profiles/rNN/hbm.json, written by tools/pmc_hbm.py from rocprofv3
    FETCH_SIZE/WRITE_SIZE passes with the gfx950 corrections), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "hbm.json")), reverse=True):
        try:
            k = json.load(open(path))["kernels"].get(symbol)
        except (OSError, ValueError, KeyError):
            continue
        if k:
            return round(k["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


PROBE_SCHEDULE = ("probed steps on one stream; the others run the encoder and decoder backward on two "
                  "streams (EngineOptions.bwd_streams)")


class one_stream:
    """The engine's backward on one stream for the block (EngineOptions.bwd_streams
    off): a probed step stamps the dominant kernel's launches, whose durations on
    two streams would include the other chain's co-running work -- the per-launch
    roofline is the kernel's own (the step's throughput is the timed region's)."""

    def __init__(self, eng):
        self.eng = eng

    def __enter__(self):
        self.prev = self.eng.opt.bwd_streams
        self.eng.opt.bwd_streams = False

    def __exit__(self, *exc):
        self.eng.opt.bwd_streams = self.prev
        return False


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        local = local % torch.cuda.device_count()  # == local on a node with a GPU per rank
        torch.cuda.set_device(local)
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    cfg = yaml.safe_load(open(os.path.join(ROOT, "vae_npvc_amd", "conf", f"{a.config}.yaml")))
    cfg["compute_dtype"] = a.dtype
    cfg["batch_size"] = B_PER_GPU
    cfg["grad_sync"] = a.grad_sync
    if os.environ.get("VQX_ENGINE"):  # A/B runs: engine schedule options as JSON (engine/step.py EngineOptions)
        cfg["engine"] = json.loads(os.environ["VQX_ENGINE"])

    from vae_npvc_amd import ops
    from vae_npvc_amd.trainer.basic import Trainer
    torch.manual_seed(777)
    np.random.seed(777)
    tr = Trainer(cfg)
    mel = cfg["encoder"]["in_channels"][0]
    gen = torch.Generator(device="cpu").manual_seed(1234 + rank)
    n_batches = 4
    xs = [torch.randn(B_PER_GPU, mel, T_FRAMES, generator=gen).to(dev) for _ in range(n_batches)]
    ys = [torch.randint(0, cfg["y_num"], (B_PER_GPU, 1), generator=gen).to(dev) for _ in range(n_batches)]

    masked = None
    if a.reserve_cus > 0:
        masked, cus_used = ops.cu_masked_stream(a.reserve_cus)
        torch.cuda.set_stream(masked)
    comm = tr.engine.comm
    for i in range(a.warmup):
        _, det = tr.train_step((xs[i % n_batches], ys[i % n_batches]))
    if a.warmup:
        dict(det)  # materialise once: surfaces any asynchronous error before timing
    probe = None if a.no_probe else ops.LaunchProbe()
    per_kernel = bool(os.environ.get("VQX_BENCH_KERNELS"))
    if probe is not None and not per_kernel:
        # one untimed probed step names the dominant kernel (most time per step);
        # the timed region then stamps only that kernel's launches (an
        # event-stamped dispatch costs ~4.6 us of queue time)
        probe.clear()
        ops.set_probe(probe)
        with one_stream(tr.engine):
            tr.train_step((xs[0], ys[0]))
        ops.set_probe(None)
        per = {}
        for sym, _, sec, _, info in probe.records():
            per.setdefault(sym, [0.0, info])[0] += sec
        probe.select(max(per.values(), key=lambda v: v[0])[1])
    if probe is not None:
        probe.clear()
    if comm is not None:  # communication diagnostics over the timed region
        comm.reset_stats()
        comm.timing = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        # the GEMM probe samples every `probe_every`-th step of the timed region
        # (an event-stamped dispatch costs ~4.6 us of queue time)
        probed = probe is not None and i % a.probe_every == a.probe_every // 2
        if probe is not None:
            ops.set_probe(probe if probed else None)
        if probed:  # a probed step runs on one stream: the stamped kernel's own duration (see one_stream)
            with one_stream(tr.engine):
                _, det = tr.train_step((xs[i % n_batches], ys[i % n_batches]))
        else:
            _, det = tr.train_step((xs[i % n_batches], ys[i % n_batches]))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ops.set_probe(None)
    summ = probe.summary() if probe is not None else None  # the timed region's probed launches
    if probe is not None:
        probe.select(None)
    elapsed = t1 - t0
    comm_out = None
    if comm is not None:
        comm.timing = False
        nbytes, calls, grad_ms, ema_ms = comm.stats()
        per = torch.tensor([nbytes / a.steps, calls / a.steps, grad_ms / a.steps, ema_ms / a.steps],
                           device=dev, dtype=torch.float64)
        allr = [torch.empty_like(per) for _ in range(world)]
        dist.all_gather(allr, per)
        allr = torch.stack(allr).cpu().tolist()
        # per rank and step: bytes all-reduced, collectives issued, and how long
        # the compute stream stood still behind the gradient all-reduces
        # (Comm.finish) and the EMA-statistics all-reduce (codebook update)
        comm_out = {"bytes_per_step": round(allr[0][0]), "collectives_per_step": allr[0][1],
                    "grad_wait_ms": [round(r[2], 4) for r in allr], "ema_wait_ms": [round(r[3], 4) for r in allr],
                    "bucket_bytes": comm.bucket * 4, "backend": comm.backend,
                    "grad_sync": "overlap" if comm.overlap else "end"}
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    detail = dict(det)
    # the same loop as a recipe runs it: the reference's bin/train.py:128-132
    # appends every loss_detail value every iteration, so each step ends in a
    # host read of the step's statistics (one device sync per step)
    read_ms = time_read_loss(tr, xs, ys, a.steps, world) if a.read_loss else None
    if world > 1 and world != a.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}; reporting n_gpus={world}", file=sys.stderr)
    frames = B_PER_GPU * T_FRAMES * world * a.steps
    value = frames / elapsed
    ms = 1e3 * elapsed / a.steps

    roof = None
    kernels = None
    if probe is not None:
        n_probed = sum(1 for i in range(a.steps) if i % a.probe_every == a.probe_every // 2)
        kernels = {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                   for k, v in summ.items()}
        dom = max(summ.items(), key=lambda kv: kv[1]["seconds"])
        name, s = dom
        peak = PEAK_BF16 if a.dtype == "bf16" else PEAK_F32
        ach = s["flops"] / s["seconds"]
        traffic, tsrc = committed_traffic(name)
        roof = {"bound": "mfma", "kernel": name, "achieved": round(ach / 1e12, 2), "peak": peak / 1e12,
                "unit": "TFLOP/s", "frac": round(ach / peak, 4), "traffic": traffic, "traffic_unit": "bytes/launch",
                "traffic_source": tsrc,
                "probed_steps": n_probed, "launches_per_step": s["launches"] / max(1, n_probed),
                "avg_launch_us": round(s["avg_us"], 2),
                "flops_per_launch": s["flops"] / s["launches"],
                "schedule": PROBE_SCHEDULE if tr.engine._bwd_concurrent() else "one stream"}

    out = {
        "metric": "mel-frames/sec/GPU VQ-VAE train step (80-dim mel, batch=64x256f) at 1/2/4/8 GPUs",
        "value": round(value, 1), "unit": "mel-frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "ms_per_step_read_loss": None if read_ms is None else round(read_ms, 3),
        "read_loss_overhead": None if read_ms is None else round(read_ms / ms - 1.0, 4),
        "dtype": a.dtype, "data": "synthetic (N(0,1) 80-mel, random speaker ids; seeded random-init weights)",
        "config": {"workload": f"{a.config} VQ-VAE (K={cfg['z_num']}, {mel}-mel), {B_PER_GPU}x{T_FRAMES} frames per GPU",
                   "global_batch": B_PER_GPU * world, "seq_len": T_FRAMES, "parallelism": f"dp{world}"},
        "step_mfma_frac": round(FLOP_PER_FRAME * value / world / (PEAK_BF16 if a.dtype == "bf16" else PEAK_F32), 4),
        "roofline": roof,
        "schedule": {"backward_streams": 2 if tr.engine._bwd_concurrent() else 1,
                     "encoder_backward_early": bool(tr.engine._bwd_concurrent() and tr.engine.opt.enc_bwd_early)},
        "loss": {k: round(v, 4) for k, v in detail.items()},
        "comm": comm_out,
    }
    if masked is not None:
        out["reserved_cus"] = {"reserved": a.reserve_cus, "cus_used": cus_used}
    vq = time_vq(tr, a.vq_reps) if a.vq_reps > 0 else None
    out["vq"] = vq
    if world == 1 and a.fp32_steps > 0 and a.dtype != "fp32":
        out["fp32"] = time_fp32(cfg, a.fp32_steps, dev)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, a.cpu_steps)
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        if kernels is not None and per_kernel:
            out["kernels"] = kernels
            if os.environ.get("VQX_BENCH_KERNELS") == "2":
                out["layers"] = {k: (v["launches"] // max(1, n_probed), round(v["avg_us"], 1), round(v["tflops"], 1))
                                 for k, v in probe.summary(by_shape=True).items()}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
