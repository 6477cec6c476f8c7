#!/bin/bash
# Same-box A/B of the in-tree library against a variant build, with the kernel
# trace of both: the kernel / step / config GPU tests on the in-tree library,
# rocprofv3 --kernel-trace of the bf16 bench on each (per-kernel times per step:
# tools/trace_steps.py gpurun_out/TAG/p_{new,old}/run_kernel_trace.csv), then
# the bench step on both, two interleaved passes (tools/gpu_lib_step_ab.sh).
# usage: bash tools/gpu_lib_trace_ab.sh TAG variant.so
TAG=${1:-libtrace}; OLD=$2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_step.py tests/test_gpu_configs.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for side in new old; do
  lib=""; [ $side = old ] && lib=$OLD
  VQX_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$side -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > $O/log_$side.txt 2>&1 || exit 1
done
bash tools/gpu_lib_step_ab.sh $TAG "$OLD"
