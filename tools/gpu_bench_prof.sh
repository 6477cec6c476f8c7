# Bench (per-layer breakdown) + rocprof kernel-trace of the same command line.
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-read-loss > $O/prof.log 2>&1 || exit $?
grep '^{' $O/bench.log | cut -c1-300
grep '^{' $O/prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('under rocprof:', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
