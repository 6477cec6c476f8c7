#!/bin/bash
# wn_bwd_kernel variants (tools/lab/wn_nf*_vpre*.so, built with
#   python -m vae_npvc_amd.csrc.build --out tools/lab/wn_nfN_vpreV.so -D VQX_WN_NF=N -D VQX_WN_VPRE=V)
# in the bf16 step, rocprofv3 kernel trace per variant (WN_LIBS="lib1.so lib2.so ...")
set -o pipefail
cd "$(dirname "$0")/../.."
for lib in "" $WN_LIBS; do
  tag=wn_$(basename ${lib:-default} .so)
  VQX_LIB=$lib bash tools/gpu_prof_step.sh $tag > /dev/null || exit $?
  echo "$tag $(head -1 gpurun_out/$tag/rocprof_summary.txt) | $(grep wn_bwd gpurun_out/$tag/rocprof_summary.txt)"
done | tee gpurun_out/wn_lab.txt
