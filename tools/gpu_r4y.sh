# round-4: VQ tests after the width-parameter rename + smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q -k "vq or golden" --timeout 300 --timeout-method thread > $O/tests_vq.log 2>&1
rc=$?; echo "vq tests rc=$rc"; tail -2 $O/tests_vq.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; exit $rc
