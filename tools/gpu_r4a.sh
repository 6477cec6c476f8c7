set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-600 $O/bench.json
VQB_K=512 timeout -k 10 120 python tools/vq_bench.py 50 > $O/vq_bench.txt 2>&1 || exit $?
cat $O/vq_bench.txt
VQB_K=512 bash tools/gpu_pmc_cmd.sh r4a python3 tools/vq_bench.py 20 > $O/vq_pmc.log 2>&1 || exit $?
grep vq_forward gpurun_out/r4a/pmc/summary.txt
