# round-4 evidence: step SQ counters per kernel and the 1x1 layers' main-loop / epilogue split
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5g; mkdir -p $O
bash tools/gpu_pmc_step.sh r5g > $O/pmc_step.txt 2>&1 || { tail -20 $O/pmc_step.txt; exit 1; }
timeout -k 10 300 python3 tools/k1_breakdown.py 30 > $O/k1_breakdown.txt 2>&1 || { tail -20 $O/k1_breakdown.txt; exit 1; }
cat $O/k1_breakdown.txt
