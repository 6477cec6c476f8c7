#!/bin/bash
# Build (CPU side: bash tools/lab/k1_lab.sh build) or run (GPU box) the 1x1 GEMM lab variants.
set -o pipefail
cd "$(dirname "$0")"
V=${K1_V:-"s0m0 n3m0 n4m0 n3m3 n4m3 s0m3"}
if [ "$1" = build ]; then
  for v in $V; do
    st=${v:1:1}; md=${v:3:1}
    D="-DVQX_LAB_MODE=$md"
    [ ${v:0:1} = s ] && [ $st -ne 0 ] && D="$D -DVQX_GEMM_STAGGER=$st"
    [ ${v:0:1} = p ] && D="$D -DVQX_EPI_PREFETCH=$st"
    [ ${v:0:1} = v ] && D="$D -DVQX_EPI_PREVEC_DGRAD=$st"
    [ ${v:0:1} = g ] && D="$D -DVQX_LAB_NO_GNBWD=1"
    [ ${v:0:1} = t ] && D="$D -DVQX_LAB_GNBWD_NOTRANS=1"
    [ ${v:0:1} = r ] && D="$D -DVQX_EPI_PREFETCH_DGRAD=1"
    [ ${v:0:1} = n ] && D="$D -DK1_NST=$st"
    [ ${v:0:1} = l ] && D="$D -DVQX_EPI_PREFETCH_DGRAD=1 -DVQX_EPI_PREFETCH_LATE=$st"
    [ ${v:0:1} = f ] && D="$D -DVQX_EPI_PREFETCH_LATE=$st"
    [ ${v:0:1} = e ] && D="$D -DVQX_EPI_SLAB_PREFETCH=$st"
    /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=fast -I ../../include \
      -I ../../vae_npvc_amd/csrc $D k1_lab.cpp -o k1_lab_$v.bin &
  done
  wait
  exit 0
fi
mkdir -p ../../gpurun_out
for v in $V; do
  timeout -k 10 60 ./k1_lab_$v.bin || exit $?
done | tee ../../gpurun_out/k1_lab.txt
