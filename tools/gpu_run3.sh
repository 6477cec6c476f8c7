# Full GPU pass: parity tests, bench (per-kernel summary), rocprof kernel-trace.
# usage: bash tools/gpu_run3.sh TAG
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -rs --timeout 300 > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe > $O/prof.log 2>&1
echo "prof rc=$?" >> $O/prof.log
tail -4 $O/tests.log
grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' $O/bench.log
python3 tools/prof_summary.py $O/prof 7 25 > $O/prof_summary.txt
