#!/bin/bash
# VQ forward fixed-cost lab: variants without the score loop / epilogue (VQX_VQ_LAB), kernel durations from a
# rocprofv3 kernel trace of tools/vq_fixed.py.
# Build on the CPU side first:  for v in 1 2 3; do python -m vae_npvc_amd.csrc.build --out tools/lab/vqlab$v.so -D VQX_VQ_LAB=$v; done
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/vqlab
for v in 0 1 2 3; do
  lib=""; [ $v -ne 0 ] && lib="tools/lab/vqlab$v.so"
  env ${lib:+VQX_LIB=$lib} timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/vqlab/v$v -o run --output-format csv -- python3 tools/vq_fixed.py > gpurun_out/vqlab/v$v.log 2>&1 || exit $?
done
