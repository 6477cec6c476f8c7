#!/bin/bash
# Per-kernel probe of the fused launches at several interleave periods, same box, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/chunkp
for rep in 1 2; do
  for c in 8 128 256; do
    VQX_DUAL_CHUNK=$c VQX_BENCH_KERNELS=1 timeout -k 10 200 python -u bench.py --steps 30 --no-cpu-baseline --fp32-steps 0 \
      --vq-reps 0 --probe-every 1 > gpurun_out/chunkp/c$c.json 2> gpurun_out/chunkp/c$c.err || exit $?
    python3 -c "
import json
d = json.load(open('gpurun_out/chunkp/c$c.json'))
k = d['kernels']
f = lambda s: round(k[s]['avg_us'], 1) if s in k else None
print('chunk $c', d['ms_per_step'], 'dual_tr<4>', f('vqx::dual_tr_kernel<4>'), 'dual_tr<1>', f('vqx::dual_tr_kernel<1>'),
      'dual_k1<6>', f('vqx::dual_k1_kernel<6, true>'))"
  done
done | tee gpurun_out/chunkp/summary.txt
