# round-4: batched weight-norm backward, loads in flight a thread (NF 2 / 8 lab builds): A/B + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
L=vae_npvc_amd/lib/ab
bash tools/gpu_ab_env.sh r5c "VQX_LIB=$L/libvqx_nf2.so" "VQX_LIB=$L/libvqx_nf8.so" | tee $O/ab.txt || exit $?
for v in base nf2 nf8; do
  lib=$([ $v = base ] && echo "" || echo $L/libvqx_$v.so)
  VQX_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > $O/prof_$v.log 2>&1 || exit $?
  echo "$v $(python3 tools/trace_steps.py $O/prof_$v/run_kernel_trace.csv 40 | grep wn_bwd)"
done
