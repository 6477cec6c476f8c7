set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py -m gpu -x -v -k "aishell3" --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $O/tests.log | head -20; exit $rc
