#!/bin/bash
# Build (CPU: bash tools/lab/pp_lab.sh build) or run (GPU box) the ping-pong lab variants (VQX_PP_LAB 0..4)
set -o pipefail
cd "$(dirname "$0")"
if [ "$1" = build ]; then
  for v in 0 1 2 3 4; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -I ../../include \
      -I ../../vae_npvc_amd/csrc -DVQX_PP_LAB=$v tr_lab.cpp -o pp_lab$v.bin &
  done
  wait
  exit 0
fi
export TMPDIR=/tmp
O=../../gpurun_out/pp_lab; mkdir -p $O
for v in 0 1 2 3 4; do
  echo "== VQX_PP_LAB=$v"; TR_LAB_SKIP_WGRAD=1 timeout -k 10 60 ./pp_lab$v.bin || exit $?
done > $O/times.txt
cd ../.. && bash tools/gpu_pmc_cmd.sh pp_lab tools/lab/pp_lab0.bin > /dev/null
