# round-4 A/B: VQ store rotation (in-tree) vs not; bf16 vs fp32 split-K slabs on the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
for pass in 0 1; do
  for lib in "" tools/lab/var/libvqx_norot.so; do
    echo "== pass $pass lib=${lib:-in-tree}"
    env ${lib:+VQX_LIB=$lib} VQB_K=512 timeout -k 10 120 python tools/vq_bench.py 100 2>&1 | grep 'K=' || exit $?
  done
done | tee $O/vq_ab.txt
bash tools/gpu_ab_env.sh r4b "VQX_SLAB_F32=1" | tee $O/slab_ab.txt
