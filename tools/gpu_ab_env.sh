#!/bin/bash
# Same-box A/B of one environment switch on the bf16 bench step:
#   bash tools/gpu_ab_env.sh NAME VAR VALUE_A VALUE_B   (alternating A B A B, 20 steps each)
set -o pipefail
cd "$(dirname "$0")/.."
NAME=$1; VAR=$2; A=$3; B=$4
mkdir -p gpurun_out/ab_$NAME
for v in $A $B $A $B; do
  env $VAR=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp32-steps 0 \
    --vq-reps 0 --no-probe > gpurun_out/ab_$NAME/b_$v.json 2> gpurun_out/ab_$NAME/b_$v.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$NAME/b_$v.json'));print('$VAR=$v', d['ms_per_step'], d['value'])"
done | tee gpurun_out/ab_$NAME/summary.txt
