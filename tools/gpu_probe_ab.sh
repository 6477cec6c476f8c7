# bench with and without the in-loop GEMM probe (the probe must not perturb `value`)
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/pa_probe$i.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --no-probe > gpurun_out/pa_noprobe$i.log 2>&1 || exit $?
done
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/pa_probe*.log gpurun_out/pa_noprobe*.log
