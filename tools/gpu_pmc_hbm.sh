# HBM bytes per dispatch: two separate --pmc passes (no trace domains), then the summary.
# usage: bash tools/gpu_pmc_hbm.sh TAG
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG/pmc
mkdir -p $O
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-read-loss --no-probe --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-read-loss --no-probe --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/write.log 2>&1 || exit $?
python3 tools/pmc_hbm.py $O 31330720 $O/hbm.json
