# tap-reuse L2 prefetch lab (round 6, profiles/r06/tr_prefetch_ab.txt).  Variants: git apply
# tools/lab/tr_prefetch.patch, then python -m vae_npvc_amd.csrc.build --out lab_so/pfN.so -D VQX_TR_PF=N (N = 1, 2)
set -o pipefail
mkdir -p gpurun_out/pf
VQX_LIB=lab_so/pf2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "tap_reuse or fused_dgrad" > gpurun_out/pf/t.log 2>&1 || { tail -5 gpurun_out/pf/t.log; exit 1; }
tail -1 gpurun_out/pf/t.log
for v in "" lab_so/pf1.so lab_so/pf2.so; do
  tag=pf/tr_$(basename ${v:-base} .so)
  VQX_LIB=$v bash tools/gpu_prof_step.sh $tag > /dev/null || exit 1
  echo "$tag $(python3 tools/trace_steps.py gpurun_out/$tag/prof/run_kernel_trace.csv 60 | grep -E 'kernel time|conv_tr_kernel<0, 5|dual_tr|conv_pp' | tr '\n' '|')"
done
bash tools/gpu_lib_step_ab.sh pf/ab lab_so/pf1.so lab_so/pf2.so
