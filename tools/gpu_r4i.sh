# round-4: triple-launch tests; GPU suite (in-tree lib, then the GNBWD one-pass-ahead
# variant); A/B default vs ahead lib vs tail_wgrad_1x1 off; per-XCD CU reserve; per-layer bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
AHEAD=vae_npvc_amd/lib/ab/libvqx_ahead.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "triple or fused" --timeout 200 --timeout-method thread > $O/tests_triple.log 2>&1
rc=$?; echo "triple tests rc=$rc"; tail -2 $O/tests_triple.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VQX_LIB=$AHEAD timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_ahead.log 2>&1
rc=$?; echo "pytest ahead rc=$rc"; tail -3 $O/tests_ahead.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4i "VQX_LIB=$AHEAD" 'VQX_ENGINE={"tail_wgrad_1x1":false}' | tee $O/ab.txt || exit $?
for r in 0 8 16 32 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 --reserve-cus $r > $O/bench_res$r.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_res$r.json')); print('reserve $r', d['value'], d['ms_per_step'], d.get('reserved_cus'))"
done | tee $O/cu_reserve.txt || exit $?
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > $O/bench_layers.json 2> $O/bench_layers.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_layers.json')); print(d['value'], d['ms_per_step'])
for k,v in sorted(d['layers'].items(), key=lambda kv: -kv[1][0]*kv[1][1])[:16]: print('  ', k, v)
"
