# Weight-norm backward at 64 VGPRs (wave-per-row path one column group per lane: 8 waves/SIMD)
# vs the 86-VGPR build (tools/lab/wn_occ_old.so, 5 waves/SIMD); same box.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/wnocc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_step.py tests/test_gpu_configs.py > gpurun_out/wnocc/tests.log 2>&1; rc=$?; tail -1 gpurun_out/wnocc/tests.log; [ $rc -eq 0 ] || exit $rc
for lib in "" tools/lab/wn_occ_old.so; do
  VQX_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wnocc/p_${lib:+old} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > gpurun_out/wnocc/log_${lib:+old}.txt 2>&1 || exit 1
done
bash tools/gpu_lib_step_ab.sh wnocc tools/lab/wn_occ_old.so
