# round-4: dead-code row ids passed to the gather kernel by value -- suites, trace, A/B against the previous tree (ab_base/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_rccl.py tests/test_gpu_ddp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for pass in 0 1; do
  for v in base new base new; do
    d=$([ $v = base ] && echo ab_base || echo .)
    (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40) > $O/ab_${pass}_$v.json 2> $O/ab_${pass}_$v.err || exit $?
    echo "pass $pass $v $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" $O/ab_${pass}_$v.json)"
  done
done | tee $O/ab.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 --no-probe > $O/prof.log 2>&1 || exit $?
