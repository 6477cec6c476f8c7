# round-4: GroupNorm backward apply with 8 channels (16-B accesses) a thread (lab build) --
# GPU suite on the variant, A/B, kernel trace of the variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4q; mkdir -p $O
V=vae_npvc_amd/lib/ab/libvqx_gnw8.so
VQX_LIB=$V timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4q "VQX_LIB=$V" | tee $O/ab.txt || exit $?
VQX_LIB=$V timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/prof.log 2>&1 || exit $?
python3 tools/trace_steps.py $O/prof/run_kernel_trace.csv 14
