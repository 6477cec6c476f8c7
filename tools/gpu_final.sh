#!/bin/bash
# Round records on the final tree (profiles/rNN): part 1 = the GPU suite, smoke,
# the default bench line (with CPU baseline) and a kernel trace of the bench
# (rocprof_summary.txt via tools/trace_steps.py); part 2 = HBM bytes per launch
# (FETCH_SIZE / WRITE_SIZE passes), memory-pipeline counters of one step
# (tools/pmc_units.sh) and the CU-reservation cost (--reserve-cus 0 / 8, two
# interleaved passes).  usage: bash tools/gpu_final.sh TAG 1|2
TAG=${1:-final}; PART=${2:-1}
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
if [ "$PART" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
  cut -c1-300 $O/bench.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py \
    --no-cpu-baseline --no-read-loss > $O/prof.log 2>&1 || exit 1
  python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv 45 > $O/rocprof_summary.txt && head -14 $O/rocprof_summary.txt
  # the one-stream schedule the bench's probed steps use (the roofline kernel's own launch durations)
  VQX_ENGINE='{"bwd_streams": false}' timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof1 -o run \
    --output-format csv -- python3 bench.py --no-cpu-baseline --no-read-loss > $O/prof1.log 2>&1 || exit 1
  python3 tools/trace_steps.py $O/prof1/run_kernel_trace.csv 45 > $O/rocprof_summary_one_stream.txt && head -4 $O/rocprof_summary_one_stream.txt
else
  bash tools/gpu_pmc_hbm.sh $TAG || exit 1
  bash tools/pmc_units.sh $TAG python3 bench.py --steps 2 --warmup 1 --no-read-loss --no-probe --no-cpu-baseline \
    --fp32-steps 0 --vq-reps 0 > /dev/null || exit 1
  for pass in 0 1; do
    for r in 0 8; do
      timeout -k 10 300 python bench.py --reserve-cus $r --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 \
        --no-read-loss > $O/cu_${pass}_$r.json 2> $O/cu_${pass}_$r.err || exit 1
      echo "pass $pass reserve $r $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" $O/cu_${pass}_$r.json)"
    done
  done | tee $O/cu_reserve.txt
fi
