#!/bin/bash
# Memory-pipeline counters per kernel of any python command: three separate
# --pmc passes (no trace domains), summarised by tools/pmc_units.py.
#   pass 1: TA / TD busy and stall cycles, MFMA busy, wave cycles
#   pass 2: L1 (TCP) -> L2 requests and stalls, LDS-DMA wavefronts
#   pass 3: L2 (TCC) hits / misses / requests, L1 -> L2 read latency
# usage: bash tools/pmc_units.sh TAG python3 script.py args...
TAG=$1; shift
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG/units
mkdir -p $O
timeout -s KILL 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $O/p1 -o run --output-format csv -- "$@" > $O/p1.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_READ_LDS_WAVEFRONTS_sum GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- "$@" > $O/p2.log 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE -d $O/p3 -o run --output-format csv -- "$@" > $O/p3.log 2>&1 || exit $?
python3 tools/pmc_units.py $O > $O/summary.txt
cat $O/summary.txt
