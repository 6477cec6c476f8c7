#!/bin/bash
# round 2: new config tests + DDP vs golden + trainer loop, then the bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -s > gpurun_out/r02a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r02a_bench.json 2> gpurun_out/r02a_bench.err
echo "bench rc=$?"
