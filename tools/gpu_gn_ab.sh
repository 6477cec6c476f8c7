#!/bin/bash
# GroupNorm kernel A/B: the GN GPU tests on the in-tree library, tools/gn_bench.py on
# it and on each variant library, then the bench step on all (tools/gpu_lib_step_ab.sh).
# usage: bash tools/gpu_gn_ab.sh TAG variant.so ...
TAG=${1:-gnab}; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "glu or gn" > gpurun_out/$TAG/tests.log 2>&1; rc=$?; tail -2 gpurun_out/$TAG/tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 0 1; do
  for lib in "" "$@"; do echo "[${lib:-in-tree}]"; VQX_LIB="$lib" timeout -k 10 120 python tools/gn_bench.py 200 | tail -1 || exit 1; done
done
bash tools/gpu_lib_step_ab.sh $TAG "$@"
