# round-4: GPU suite + per-layer bench + bench line + CU-reserve runs (what co-resident RCCL work costs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > $O/bench_layers.json 2> $O/bench_layers.err || exit $?
python3 -c "
import json; d=json.load(open('$O/bench_layers.json')); print(d['value'], d['ms_per_step'])
for k,v in sorted(d['layers'].items(), key=lambda kv: -kv[1][0]*kv[1][1])[:14]: print('  ', k, v)
"
for r in 0 16 32 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 --reserve-cus $r > $O/bench_res$r.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_res$r.json')); print('reserve $r', d['value'], d['ms_per_step'], d.get('reserved_cus'))"
done | tee $O/cu_reserve.txt
