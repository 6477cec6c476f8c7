# GPU tests, then bench A/B over an env setting: bash tools/gpu_ab_env.sh TAG "VAR=a" "VAR=b" ...
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NO_TESTS" ]; then timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi; fi
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$i.log 2>&1 || exit $?
  echo "$kv: $(grep '^{' $O/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
