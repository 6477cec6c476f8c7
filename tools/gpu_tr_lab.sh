#!/bin/bash
# Lab A/B of the 3-tap FWD kernel variants (build.py -D VQX_TR_FWD_LAB=n):
# the isolated encoder k3 FWD with GroupNorm statistics (tools/gemm_bench.py),
# two interleaved passes per library, then the bench step on each library.
# usage: bash tools/gpu_tr_lab.sh TAG lib1.so ...
TAG=${1:-trlab}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
for pass in 0 1; do
  for lib in "" "$@"; do
    echo "pass $pass [${lib:-in-tree}] $(VQX_LIB="$lib" timeout -k 10 120 python tools/gemm_bench.py --only enc_k3_fwd --gnstats --iters 100 --rotate 4 2>/dev/null | tail -1)"
  done
done | tee $O/micro.txt
bash tools/gpu_lib_step_ab.sh $TAG "$@"
