# SQ counters of the train step (two separate --pmc passes, no trace domains), summarised per kernel.
# usage: bash tools/gpu_pmc_step.sh TAG
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG/pmc
mkdir -p $O
P="python3 bench.py --steps 2 --warmup 1 --no-probe --no-cpu-baseline --fp32-steps 0 --vq-reps 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/p1 -o run --output-format csv -- $P > $O/p1.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- $P > $O/p2.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
