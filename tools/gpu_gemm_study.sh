# GEMM study: isolated layer timings, hipBLASLt yardstick, PMC stall breakdown.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gstudy
mkdir -p $O
timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm.log 2>&1 || exit $?
VQX_GEMM_SUB=2 timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm_sub2.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/blas_ref.py > $O/blas.log 2>&1 || exit $?
bash tools/gpu_gemm_pmc.sh || exit $?
cp -r gpurun_out/gpmc $O/
