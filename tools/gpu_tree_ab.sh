cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sess_ab
for pass in 0 1; do
  (cd ab_old && timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > ../gpurun_out/sess_ab/old_$pass.json 2>/dev/null) || exit 1
  echo "pass $pass [926b24d] $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" gpurun_out/sess_ab/old_$pass.json)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --steps 40 > gpurun_out/sess_ab/new_$pass.json 2>/dev/null || exit 1
  echo "pass $pass [HEAD] $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']), d['ms_per_step'])" gpurun_out/sess_ab/new_$pass.json)"
done
