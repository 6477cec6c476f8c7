#!/bin/bash
# SQ counters of any python command (two separate --pmc passes, no trace domains), summarised per kernel.
# usage: bash tools/gpu_pmc_cmd.sh TAG python3 script.py args...
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG/pmc
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $O/p1 -o run --output-format csv -- "$@" > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- "$@" > $O/p2.log 2>&1 || exit $?
python3 tools/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
