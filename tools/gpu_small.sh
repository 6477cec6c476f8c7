#!/bin/bash
# Kernel tests of the optimizer / GN-GLU / fused GEMM launches, then a per-step rocprof trace of the bf16 bench step.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/small
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "adam or fused_dgrad_wgrad or gn_glu or gn_bwd or gnbwd" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 \
  --warmup 5 --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/prof.log 2>&1 || exit $?
grep '^{' $O/prof.log | cut -c1-220
python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv 16
