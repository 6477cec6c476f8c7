#!/bin/bash
# A/B of environment settings on the bench line, interleaved over two passes so
# clock drift cancels: tools/gpu_ab_env.sh TAG "K1=a K2=b" "K1=c" ...
# (the empty setting -- the defaults -- always runs first in each pass).
# Engine schedule options go in as compact JSON, e.g. 'VQX_ENGINE={"slab_f32":true}'
# (bench.py -> Model arch "engine"), a variant library as VQX_LIB=path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-ab}; shift
O=gpurun_out/$TAG; mkdir -p $O
for pass in 0 1; do
  i=0
  for e in "" "$@"; do
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 \
      > $O/ab${pass}_$i.json 2> $O/ab${pass}_$i.err || exit $?
    echo "pass $pass [$e] $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" $O/ab${pass}_$i.json)"
    i=$((i+1))
  done
done
