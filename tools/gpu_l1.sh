set -o pipefail
bash tools/gpu_tr_lab.sh l1 lab_so/tr_r3.so lab_so/tr_r2.so || exit 1
bash tools/gpu_ab_engine.sh l1/es '{"early_stats":false}' || exit 1
for f in gpurun_out/l1/es/ab*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step'], d['ms_per_step_read_loss'])" $f; done
VQX_ENGINE='{"wgrad_fixup":true}' bash tools/gpu_prof_step.sh l1/fixon > /dev/null || exit 1
bash tools/gpu_prof_step.sh l1/fixoff > /dev/null || exit 1
head -16 gpurun_out/l1/fixon/rocprof_summary.txt; head -16 gpurun_out/l1/fixoff/rocprof_summary.txt
