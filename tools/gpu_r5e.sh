# round-4: weight-norm backward batched in chunks under data parallelism -- the step / DDP / RCCL suites
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_rccl.py tests/test_gpu_ddp.py tests/test_gpu_step.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
