# rocprofv3 kernel-trace summary of a short bench run (bf16, config 2)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/prof/bench.log 2>&1
echo "rc=$?" >> gpurun_out/prof/bench.log
