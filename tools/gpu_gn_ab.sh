timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "glu or gn" > gpurun_out/gn2.log 2>&1; rc=$?; tail -2 gpurun_out/gn2.log; [ $rc -eq 0 ] || exit $rc
for lib in "" tools/lab/gn_v1.so tools/lab/gn_old.so; do echo "[${lib:-in-tree}]"; VQX_LIB="$lib" timeout -k 10 120 python tools/gn_bench.py 200 || exit 1; done
bash tools/gpu_lib_step_ab.sh gnab2 tools/lab/gn_v1.so tools/lab/gn_old.so
