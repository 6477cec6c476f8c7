#!/bin/bash
# Same-box A/B of library builds on the bf16 bench step only (VQX_LIB=path; "" = the
# in-tree libvqx.so), two interleaved passes, 40 steps each.
# usage: bash tools/gpu_lib_step_ab.sh TAG lib1.so ...
TAG=${1:-libstep}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for pass in 0 1; do
  i=0
  for lib in "" "$@"; do
    VQX_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 \
      > $O/b_${pass}_$i.json 2> $O/b_${pass}_$i.err || exit 1
    echo "pass $pass [${lib:-in-tree}] $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" $O/b_${pass}_$i.json)"
    i=$((i+1))
  done
done
