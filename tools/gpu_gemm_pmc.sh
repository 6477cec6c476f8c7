# PMC stall breakdown of the conv GEMM on isolated config-2 shapes (separate passes, no trace domains).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gpmc
mkdir -p $O
P="python3 tools/gemm_bench.py --iters 5"
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/p1 -o run --output-format csv -- $P > $O/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- $P > $O/p2.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O
