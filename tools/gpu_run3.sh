cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -q -rs --timeout 300 > gpurun_out/t6.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t6.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VQX_BENCH_KERNELS=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench6.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench6.log
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/prof6
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-probe > gpurun_out/prof6/bench.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof6/bench.log
