# round-4: GPU suite; A/B weight-norm backward 16-B bf16 slab loads (default) vs 8-B (VQX_WN16=0)
# vs 16-B with 8 loads in flight; kernel trace of the default step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
L=vae_npvc_amd/lib/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4m "VQX_LIB=$L/libvqx_wn8.so" "VQX_LIB=$L/libvqx_wnnf8.so" | tee $O/ab.txt || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/prof.log 2>&1 || exit $?
python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv 16
