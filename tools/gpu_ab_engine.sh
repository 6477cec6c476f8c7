#!/bin/bash
# Same-box A/B of engine options on the bf16 bench step: defaults first, then
# each VQX_ENGINE JSON given, two interleaved passes, 40 steps each.
# usage: bash tools/gpu_ab_engine.sh TAG '{"kernel_policy":5}' ...
TAG=${1:-ab}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for pass in 0 1; do
  i=0
  for e in "" "$@"; do
    VQX_ENGINE="$e" timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 \
      > $O/ab${pass}_$i.json 2> $O/ab${pass}_$i.err || exit 1
    echo "pass $pass [${e:-defaults}] $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" $O/ab${pass}_$i.json)"
    i=$((i+1))
  done
done
