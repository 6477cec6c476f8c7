#!/bin/bash
# quick loop: the GPU tests matching $1 (pytest -k), then the step profile (TAG $2)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k "$1" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -2 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_prof_step.sh $2 > /dev/null || exit $?
head -12 gpurun_out/$2/rocprof_summary.txt
