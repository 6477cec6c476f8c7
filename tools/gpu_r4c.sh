# round-4 A/B: 1x1 WGRAD first in the dual launch with fewer splits, fp32 vs bf16 slabs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "dual or fused" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VQX_K1_WFIRST=1 VQX_SLAB_F32=1 VQX_WGRAD_WGS_1X1=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -k "bench_step" --timeout 200 --timeout-method thread > $O/tests2.log 2>&1
rc=$?; echo "tests2 rc=$rc"; tail -2 $O/tests2.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4c "VQX_SLAB_F32=1" "VQX_K1_WFIRST=1 VQX_SLAB_F32=1 VQX_WGRAD_WGS_1X1=128" "VQX_K1_WFIRST=1 VQX_SLAB_F32=1 VQX_WGRAD_WGS_1X1=256" "VQX_K1_WFIRST=1 VQX_WGRAD_WGS_1X1=128" "VQX_SLAB_F32=1 VQX_WGRAD_WGS_1X1=128" | tee $O/ab.txt
