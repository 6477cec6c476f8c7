# round-4: GPU suite (GN forward/backward apply with early row loads); A/B 1x1 FWD/DGRAD grid
# stagger variants (lab builds); kernel trace of the default step (GN kernel times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
L=vae_npvc_amd/lib/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4l "VQX_LIB=$L/libvqx_s2.so" "VQX_LIB=$L/libvqx_s4.so" "VQX_LIB=$L/libvqx_s4r1.so" "VQX_LIB=$L/libvqx_s7.so" | tee $O/ab.txt || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/prof.log 2>&1 || exit $?
python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv 24
