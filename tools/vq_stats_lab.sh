#!/bin/bash
# EMA-statistics kernel lab (VQX_STATS_LAB variants built as tools/lab/stlab$v.so), kernel trace of tools/vq_bench.py K=512
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/stlab
for v in 0 1 2 4 7; do
  lib=""; [ $v -ne 0 ] && lib="tools/lab/stlab$v.so"
  env ${lib:+VQX_LIB=$lib} VQB_K=512 VQB_E=randn timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/stlab/v$v -o run --output-format csv -- python3 tools/vq_bench.py 20 > gpurun_out/stlab/v$v.log 2>&1 || exit $?
done
