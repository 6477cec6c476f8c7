#!/bin/bash
# round-3 measurements: VQ N-sweep and the 1x1 breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03p
timeout -k 10 300 python tools/k1_breakdown.py 30 > gpurun_out/r03p/k1_breakdown.txt 2>&1 || exit $?
timeout -k 10 400 python tools/vq_sweep.py --reps 20 --out gpurun_out/r03p/vq_sweep.jsonl > gpurun_out/r03p/vq_sweep.log 2>&1
