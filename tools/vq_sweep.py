"""SURVEY §8d VQ sweep: vqx_vq_forward (distance, first-min argmin; the
commitment partials) from N = 16 K to 1 M frames at K in {128, 512, 1024},
D = 128, fp32, timed with HIP events on the launch stream.

Per (N, K) one JSON line with three forms of the call:
  idx_us    idx only (no z_q stores, no statistics),
  zq_us     + z_q (fp32 and bf16 copies) and the commitment sum (the step's call without EMA statistics),
  stats_us  + the EMA statistics (the step's call),
and the rooflines of the idx-only form: algorithmic bytes = z (N*D f32) +
E (K*D f32) + idx (N int64) over 8 TB/s, FLOPs = 2*N*K*D over the 157.3 TF
fp32 MFMA peak.  Codebooks are rows of z (the step's init_emb), so the argmin
work is the step's.  Usage: python tools/vq_sweep.py [--reps 20] [--out FILE]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vae_npvc_amd import ops  # noqa: E402

HBM, F32 = 8.0e12, 157.3e12


def t_us(fn, reps):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return 1e3 * e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--N", default="16384,65536,262144,1048576")
    ap.add_argument("--K", default="128,512,1024")
    a = ap.parse_args()
    D = 128
    g = torch.Generator(device="cpu").manual_seed(0)
    out = open(a.out, "w") if a.out else None
    for N in [int(v) for v in a.N.split(",")]:
        z = torch.randn(N, D, generator=g).cuda()
        idx = torch.empty(N, dtype=torch.int64, device="cuda")
        zq = torch.empty(N, D, device="cuda")
        zqc = torch.empty(N, D, device="cuda", dtype=torch.bfloat16)
        sq = torch.zeros(1, device="cuda")
        for K in [int(v) for v in a.K.split(",")]:
            E = z[torch.randperm(N, generator=g)[:K].cuda()].contiguous()
            part = torch.empty(ops.vq_workspace(N, K, True), device="cuda")
            ema = torch.zeros(K * D + K, device="cuda")
            bs, bc = ema[:K * D].view(K, D), ema[K * D:]
            reps = max(3, a.reps * 16384 // N)
            t_idx = t_us(lambda: ops.vq_forward(z, E, idx, None, None, None, part, None, None), reps)
            t_zq = t_us(lambda: ops.vq_forward(z, E, idx, zq, zqc, sq, part, None, None), reps)
            t_st = t_us(lambda: ops.vq_forward(z, E, idx, zq, zqc, sq, part, bs, bc), reps)
            nbytes = N * D * 4 + K * D * 4 + N * 8
            flops = 2.0 * N * K * D
            s = t_idx * 1e-6
            rec = {"N": N, "K": K, "idx_us": round(t_idx, 2), "zq_us": round(t_zq, 2), "stats_us": round(t_st, 2),
                   "bytes": nbytes, "flops": flops, "hbm_GBps": round(nbytes / s / 1e9, 1),
                   "hbm_frac": round(nbytes / s / HBM, 4), "tflops": round(flops / s / 1e12, 2),
                   "mfma_f32_frac": round(flops / s / F32, 4),
                   "roofline_frac": round(max(nbytes / HBM, flops / F32) / s, 4),
                   "bound": "mfma_f32" if flops / F32 > nbytes / HBM else "hbm"}
            line = json.dumps(rec)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
            del part, ema
        del z, idx, zq, zqc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
