# round-4: lazy loss statistics (device snapshot, D2H on first read) -- suites, A/B, trace gaps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_rccl.py tests/test_gpu_ddp.py tests/test_gpu_trainer_loop.py tests/test_gpu_configs.py tests/test_gpu_inference.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab_env.sh r5l_ab 'VQX_ENGINE={"lazy_stats":false}' 'VQX_ENGINE={}' 'VQX_ENGINE={"lazy_stats":false}' | tee $O/ab.txt || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 20 > $O/prof.log 2>&1 || exit $?
