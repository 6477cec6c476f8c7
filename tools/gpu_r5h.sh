# round-4: weight-norm backward entries heaviest first -- bit identity, then A/B on the bench line + traces
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5h; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_step.py -k "schedules_are_bit" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log
bash tools/gpu_ab_env.sh r5h 'VQX_ENGINE={"wn_bwd_sort":true}' | tee $O/ab.txt || exit $?
for v in base sort; do
  eng=$([ $v = base ] && echo "{}" || echo '{"wn_bwd_sort":true}')
  VQX_ENGINE=$eng timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > $O/prof_$v.log 2>&1 || exit $?
  echo "$v $(python3 tools/trace_steps.py $O/prof_$v/run_kernel_trace.csv 40 | grep -E 'wn_bwd|kernel time')"
done
