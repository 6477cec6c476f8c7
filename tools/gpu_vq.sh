#!/bin/bash
# VQ kernel: parity tests, then the variant microbenchmark
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_step.py -k "vq or VQ or fp32 or plain or inference" > gpurun_out/vq_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/vq_bench.py > gpurun_out/vq_bench.txt 2>&1
echo "bench rc=$?"
export TMPDIR=/tmp
rm -rf gpurun_out/vqprof; mkdir -p gpurun_out/vqprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vqprof -o vq --output-format csv -- python3 tools/vq_bench.py 20 > gpurun_out/vqprof/run.log 2>&1
echo "prof rc=$?"
