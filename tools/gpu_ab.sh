# GEMM tile A/B (128-row vs 256-row) on the config-2 layer shapes, then kernel tests.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x > $O/kern.log 2>&1; rc=$?; echo "rc=$rc" >> $O/kern.log
tail -3 $O/kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
VQX_GEMM_SUB=1 timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm_sub1.log 2>&1 || exit $?
VQX_GEMM_SUB=2 timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm_sub2.log 2>&1 || exit $?
paste $O/gemm_sub1.log $O/gemm_sub2.log
