# round-4: DGRAD GroupNorm-backward epilogue with all row operands loaded at the epilogue start
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > $O/bench_layers.json 2> $O/bench_layers.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_layers.json')); print(d['value'], d['ms_per_step'])
for k,v in sorted(d['layers'].items(), key=lambda kv: -kv[1][0]*kv[1][1])[:16]: print(k, v)
"
