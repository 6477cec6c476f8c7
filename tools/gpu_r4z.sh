# round-4: weight-norm backward loads in flight (VQX_WN_NF 8) and threads per row block (VQX_WN_THREADS 512)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
L=vae_npvc_amd/lib/ab
for v in nf8; do
  VQX_LIB=$L/libvqx_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q -k "wn or weight_norm or golden" --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -1 $O/tests_$v.log; [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_ab_env.sh r4z "VQX_LIB=$L/libvqx_nf8.so" "VQX_LIB=$L/libvqx_t512.so" "VQX_LIB=$L/libvqx_nf8t512.so" | tee $O/ab.txt || exit $?
for v in base nf8 t512 nf8t512; do
  lib=$([ $v = base ] && echo "" || echo $L/libvqx_$v.so)
  VQX_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > $O/prof_$v.log 2>&1 || exit $?
  echo "$v $(python3 tools/trace_steps.py $O/prof_$v/run_kernel_trace.csv 40 | grep wn_bwd)"
done
