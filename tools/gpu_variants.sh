# GEMM pipeline variants: kernel parity tests, then per-variant isolated layer timings.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/var
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/kern.log 2>&1
rc=$?; echo "rc=$rc" >> $O/kern.log; tail -5 $O/kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 1 2 3 4; do
  VQX_GEMM_VARIANT=$v timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm_v$v.log 2>&1 || exit $?
done
paste $O/gemm_v1.log $O/gemm_v2.log $O/gemm_v3.log $O/gemm_v4.log | awk '{print $1, $2, $7, $12, $17}'
