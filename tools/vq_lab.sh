#!/bin/bash
# VQ forward fixed-cost lab: variants without the score loop / epilogue (VQX_VQ_LAB), timed by tools/vq_fixed.py.
# Build on the CPU side first:  for v in 1 2 3; do python -m vae_npvc_amd.csrc.build --out tools/lab/vqlab$v.so -D VQX_VQ_LAB=$v; done
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in 0 1 2 3; do
  lib=""; [ $v -ne 0 ] && lib="VQX_LIB=tools/lab/vqlab$v.so"
  echo "== VQX_VQ_LAB=$v" >> gpurun_out/vq_lab.txt
  env $lib timeout -k 10 120 python tools/vq_fixed.py >> gpurun_out/vq_lab.txt 2>&1 || exit $?
done
