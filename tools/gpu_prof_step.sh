#!/bin/bash
# rocprofv3 kernel-trace of the bf16 config-2 step alone (25 steps, no fp32 / VQ / CPU legs), summarised per step.
# usage: bash tools/gpu_prof_step.sh TAG [extra bench args]
TAG=${1:-x}; shift
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-read-loss --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --no-probe "$@" > $O/prof.log 2>&1 || exit $?
python3 tools/prof_summary.py $O/prof 25 40 > $O/rocprof_summary.txt
grep '^{' $O/prof.log | cut -c1-200
head -45 $O/rocprof_summary.txt
