#!/bin/bash
# Build (CPU side: bash tools/lab/tr_lab.sh build) or run (GPU box) the tap-reuse kernel lab variants.
set -o pipefail
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  for v in 0 1 2 3; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -I ../../include \
      -I ../../vae_npvc_amd/csrc -DVQX_GEMM_LAB=$v tr_lab.cpp -o tr_lab$v.bin &
  done
  wait
  exit 0
fi
mkdir -p ../../gpurun_out
for v in 0 1 2 3; do
  TR_LAB_WGRAD_ONLY=$WGRAD_ONLY timeout -k 10 60 ./tr_lab$v.bin || exit $?
done | tee ../../gpurun_out/tr_lab.txt
