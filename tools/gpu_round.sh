# Round measurement: GPU tests, bench (with CPU baseline), rocprof kernel trace, HBM PMC passes.
# usage: bash tools/gpu_round.sh TAG
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
VQX_BENCH_KERNELS=2 timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-read-loss > $O/prof.log 2>&1 || exit $?
bash tools/gpu_pmc_hbm.sh $TAG || exit $?
tail -3 $O/tests.log
grep '^{' $O/bench.log | cut -c1-400
