# round-4: 3-tap FWD GEMMs with and without the GroupNorm-statistics epilogue (isolated)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4x; mkdir -p $O
for rep in 0 1; do
timeout -k 10 120 python tools/gemm_bench.py --only _fwd --iters 100 --rotate 4 || exit $?
timeout -k 10 120 python tools/gemm_bench.py --only _fwd --iters 100 --rotate 4 --gnstats || exit $?
done | tee $O/fwd_gnstats.txt
