# round-4: tap-reuse WGRAD tile order (column-tile-major runs per XCD, lab build) -- GPU suite
# on the variant, A/B, per-layer bench and FETCH_SIZE of both
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
V=vae_npvc_amd/lib/ab/libvqx_tnmaj.so
VQX_LIB=$V timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab_env.sh r4n "VQX_LIB=$V" | tee $O/ab.txt || exit $?
for lib in "" "$V"; do
  tag=$([ -z "$lib" ] && echo base || echo tnmaj)
  VQX_LIB=$lib VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > $O/layers_$tag.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('$O/layers_$tag.json')); print('$tag', d['value'], d['ms_per_step'])
for k,v in d['layers'].items():
  if 'dual_tr' in k or 'wgrad_tr' in k: print('  ', k, v)
"
  VQX_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$tag -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-probe --no-cpu-baseline --fp32-steps 0 --vq-reps 0 > $O/fetch_$tag.log 2>&1 || exit $?
  python3 - <<PY
import csv, glob, collections
f = glob.glob('$O/fetch_$tag/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'dual_tr' in r['Kernel_Name'] or 'wgrad_tr' in r['Kernel_Name']:
        acc[r['Kernel_Name']].append(float(r['Counter_Value']))
for k, v in acc.items(): print('   $tag FETCH', k, len(v), 'launches, read MB/launch (x2 gfx950 corr.):', round(2 * 1024 * sum(v) / len(v) / 1e6, 2))
PY
done
