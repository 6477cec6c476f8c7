# round-4: weight-norm table chunk 256 -- chunking test, weight-norm tests, golden steps, bench A/B-free line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q -k "weight_norm or wn or golden or chunks" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > $O/prof.log 2>&1 || exit $?
python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv 40 | grep -E "kernel time|wn_bwd"
