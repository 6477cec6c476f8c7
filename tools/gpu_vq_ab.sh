#!/bin/bash
# VQ forward A/B: the VQ kernel tests on the in-tree library, then
# tools/vq_bench.py on the in-tree library and on each variant library,
# interleaved over two passes.  Usage: tools/gpu_vq_ab.sh TAG variant.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-vqab}; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "vq or VQ" \
  > $O/tests.log 2>&1
rc=$?; echo "vq tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 0 1; do
  for lib in "" "$@"; do
    echo "== pass $pass lib=${lib:-in-tree}"
    env ${lib:+VQX_LIB=$lib} VQB_E=randn timeout -k 10 120 python tools/vq_bench.py 100 2>&1 | grep 'K=' || exit $?
  done
done | tee $O/ab.txt
