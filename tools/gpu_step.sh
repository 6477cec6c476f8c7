#!/bin/bash
# One development round trip on the GPU box: the named test files first (each
# step under its own time limit; stop at the first failure), then the whole GPU
# suite, the bench line with per-layer probe timings, and a rocprofv3 kernel
# trace of the same bench command.  Usage: tools/gpu_step.sh TAG [test files...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-x}; shift
O=gpurun_out/$TAG; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" > $O/first.log 2>&1
  rc=$?; echo "first rc=$rc"; tail -5 $O/first.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/prof.log 2>&1 || exit $?
python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv > $O/trace_summary.txt 2>&1; head -24 $O/trace_summary.txt
