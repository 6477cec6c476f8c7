cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_step.py -q -rs --timeout 300 > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VQX_BENCH_KERNELS=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench2.log
