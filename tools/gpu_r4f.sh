# round-4 A/B: s_setprio(1) around every MFMA cluster (variant library) vs the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
bash tools/gpu_ab_env.sh r4f "VQX_LIB=tools/lab/var/libvqx_prio.so" | tee $O/ab.txt
for lib in "" tools/lab/var/libvqx_prio.so; do
  env ${lib:+VQX_LIB=$lib} VQX_BENCH_KERNELS=2 timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > $O/layers_${lib:+prio}.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('$O/layers_${lib:+prio}.json')); print('lib=${lib:-default}', d['value'], d['ms_per_step'])
for k,v in sorted(d['layers'].items(), key=lambda kv: -kv[1][0]*kv[1][1])[:10]: print('  ', k, v)
"
done
