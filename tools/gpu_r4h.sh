# round-4: CU-mask -> CU mapping; triple-launch tests; GPU suite; A/B tail_wgrad_1x1 on vs off; per-layer bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 60 tools/lab/cu_map.bin | tee $O/cu_map.txt || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "triple or fused" --timeout 200 --timeout-method thread > $O/tests_triple.log 2>&1
rc=$?; echo "triple tests rc=$rc"; tail -2 $O/tests_triple.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4h 'VQX_ENGINE={"tail_wgrad_1x1":false}' 'VQX_ENGINE={"wgrad_wgs_1x1_tail":256}' | tee $O/ab.txt
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > $O/bench_layers.json 2> $O/bench_layers.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_layers.json')); print(d['value'], d['ms_per_step'])
for k,v in sorted(d['layers'].items(), key=lambda kv: -kv[1][0]*kv[1][1])[:16]: print('  ', k, v)
"
