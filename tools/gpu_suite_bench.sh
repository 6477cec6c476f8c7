#!/bin/bash
# the whole GPU suite + smoke (tools/gpu_all.sh), then a default bench line and a short rocprof step profile
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${1:-x}
bash tools/gpu_all.sh || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cut -c1-400 gpurun_out/bench_$TAG.json
bash tools/gpu_prof_step.sh $TAG > /dev/null || exit $?
head -25 gpurun_out/$TAG/rocprof_summary.txt
