# round-4: bench.py two-rank path (gloo on one GPU) and the RCCL world-1 test (grad_sync both ways)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_rccl.py -m gpu -x -v -k "bench_two_ranks or rccl" --timeout 700 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" $O/tests.log | tail -8; exit $rc
