#!/bin/bash
# Same-box A/B of the 1x1 kernel policy (0: automatic, 5: three workgroups per
# CU) at CU reserve 0 and 8 (bench.py --reserve-cus: 8 CUs masked off, a model
# of RCCL's kernels beside the GEMMs), two interleaved passes, 40 steps each.
# usage: bash tools/gpu_policy_ab.sh TAG
TAG=${1:-pol}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for pass in 0 1; do
 for pol in 0 5; do
  for res in 0 8; do
   VQX_ENGINE="{\"kernel_policy\":$pol}" timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 \
     --steps 40 --reserve-cus $res > $O/b_${pass}_${pol}_${res}.json 2> $O/b_${pass}_${pol}_${res}.err || exit 1
   echo "pass $pass policy $pol reserve $res $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" $O/b_${pass}_${pol}_${res}.json)"
  done
 done
done
