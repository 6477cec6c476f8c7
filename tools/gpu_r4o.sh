# round-4: bf16 split-K slab rounding vs fp32 slabs at full size (gradient tensors vs the fp32 step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q -s -k "slab_rounding or tracks_fp32_at_full_size" --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "full-size|passed|failed|Error" $O/tests.log; exit $rc
