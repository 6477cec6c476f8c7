# Weight-norm backward: bf16 slab sums of two column groups per pass (buffer loads) vs one (tools/lab/wn2_old.so)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wn2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_configs.py > gpurun_out/wn2/tests.log 2>&1; rc=$?; tail -1 gpurun_out/wn2/tests.log; [ $rc -eq 0 ] || exit $rc
for lib in "" tools/lab/wn2_old.so; do
  VQX_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wn2/p_${lib:+old} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > gpurun_out/wn2/log_${lib:+old}.txt 2>&1 || exit 1
done
bash tools/gpu_lib_step_ab.sh wn2 tools/lab/wn2_old.so
