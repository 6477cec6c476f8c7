#!/bin/bash
# conv_tr8_kernel (tall tap-reuse) parity, then a same-box A/B of the bf16 step:
# VQX_TR8=0 (128-frame tap reuse only) vs automatic, with per-layer probe timings.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tr8
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "tap_reuse" > gpurun_out/tr8/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tr8/tests.log
[ $rc -ne 0 ] && exit $rc
for v in 0 auto 0 auto; do
  if [ $v = auto ]; then unset VQX_TR8; else export VQX_TR8=$v; fi
  VQX_BENCH_KERNELS=2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --fp32-steps 0 \
    --vq-reps 0 > gpurun_out/tr8/bench_$v.json 2> gpurun_out/tr8/bench_$v.err || exit $?
  python3 -c "import json,sys;d=json.load(open('gpurun_out/tr8/bench_$v.json'));print('$v', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  cp gpurun_out/tr8/bench_$v.json gpurun_out/tr8/bench_${v}_$RANDOM.json
done
