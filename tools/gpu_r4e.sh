# round-4: weight-gradient GEMM time vs split count (long-K workgroups for a batched WGRAD launch)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python tools/gemm_bench.py --sweep-splits 1,2,4,8,16,32 --iters 20 2>&1 | grep -v amdgpu.ids | tee $O/wgrad_splits.txt
