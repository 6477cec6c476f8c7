# round-4: GPU suite (in-tree lib, then the GNBWD one-pass-ahead variant); A/B default vs ahead;
# per-layer bench with 1 CU per XCD reserved vs none (which kernels pay for a lost slot)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
AHEAD=vae_npvc_amd/lib/ab/libvqx_ahead.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VQX_LIB=$AHEAD timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_ahead.log 2>&1
rc=$?; echo "pytest ahead rc=$rc"; tail -3 $O/tests_ahead.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4j "VQX_LIB=$AHEAD" | tee $O/ab.txt || exit $?
for r in 0 8; do
  VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 --reserve-cus $r > $O/bench_layers_res$r.json 2> $O/bench_layers_res$r.err || exit $?
  python3 -c "
import json; d=json.load(open('$O/bench_layers_res$r.json')); print('reserve $r', d['value'], d['ms_per_step'])
for k,v in sorted(d['layers'].items(), key=lambda kv: -kv[1][0]*kv[1][1])[:18]: print('  ', k, v)
"
done | tee $O/layers_res.txt
