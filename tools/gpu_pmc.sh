cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 python3 tools/gemm_bench.py > gpurun_out/pmc/gemm_plain.log 2>&1 || exit $?
P="python3 tools/gemm_bench.py --iters 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/kt -o run --output-format csv -- $P > gpurun_out/pmc/kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d gpurun_out/pmc/p1 -o run --output-format csv -- $P > gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc/p2 -o run --output-format csv -- $P > gpurun_out/pmc/p2.log 2>&1 || exit $?
echo done
