# A/B of the GEMM staging variants, warm and rotating (cold) operands.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm_dma.log 2>&1 || exit $?
VQX_GEMM_STAGING=reg timeout -k 10 120 python3 tools/gemm_bench.py > $O/gemm_reg.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/gemm_bench.py --rotate 8 > $O/gemm_dma_cold.log 2>&1 || exit $?
VQX_GEMM_STAGING=reg timeout -k 10 200 python3 tools/gemm_bench.py --rotate 8 > $O/gemm_reg_cold.log 2>&1 || exit $?
paste $O/gemm_reg.log $O/gemm_dma.log
paste $O/gemm_reg_cold.log $O/gemm_dma_cold.log
