#!/bin/bash
# full GPU suite, then the bench with per-layer probe timings (twice)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  VQX_BENCH_KERNELS=2 timeout -k 10 200 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/bench_$r.json 2> $O/bench_$r.err || exit $?
done
