#!/bin/bash
# Same-box A/B of several environment settings on the bf16 bench step, alternating, 30 steps each:
#   bash tools/gpu_ab_multi.sh NAME "VAR=a VAR2=b" "VAR=c" ...   (an empty string = defaults)
set -o pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p gpurun_out/ab_$NAME
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp32-steps 0 \
      --vq-reps 0 --no-probe > gpurun_out/ab_$NAME/b_$i.json 2> gpurun_out/ab_$NAME/b_$i.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$NAME/b_$i.json'));print('[$cfg]', d['ms_per_step'], d['value'])"
  done
done | tee gpurun_out/ab_$NAME/summary.txt
