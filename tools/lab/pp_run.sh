#!/bin/bash
# GPU box: tap-reuse kernel lab (pp_lab0.bin) with the output check, then timing only (twice)
set -o pipefail
cd "$GRAFT_REPO_ROOT/tools/lab"
mkdir -p ../../gpurun_out
TR_LAB_SKIP_WGRAD=1 TR_LAB_CHECK=1 timeout -k 10 120 ./pp_lab0.bin > ../../gpurun_out/pp_lab_check.txt 2>&1 || { cat ../../gpurun_out/pp_lab_check.txt; exit 1; }
TR_LAB_SKIP_WGRAD=1 timeout -k 10 120 ./pp_lab0.bin > ../../gpurun_out/pp_lab.txt 2>&1 &&
TR_LAB_SKIP_WGRAD=1 timeout -k 10 120 ./pp_lab0.bin >> ../../gpurun_out/pp_lab.txt 2>&1
