#!/bin/bash
# GN-GLU forward frames-per-workgroup A/B (VQX_GLU_FPB 4/8/16/32/64): GN/GLU tests
# under each setting, then per-kernel times from a rocprofv3 --stats run each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/glu
mkdir -p $O
for f in 4 8; do
  VQX_GLU_FPB=$f timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "glu or gn or step" > $O/t$f.log 2>&1 || { tail -30 $O/t$f.log; exit 1; }
  tail -1 $O/t$f.log
done
for f in 16 8 4 16 8 4; do
  VQX_GLU_FPB=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p$f -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --no-probe --steps 20 --warmup 5 > $O/b$f.json 2> $O/b$f.err || exit $?
  python3 - $O/p$f/run_kernel_stats.csv $f $O/b$f.json <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
d = json.load(open(sys.argv[3]))
for r in rows:
    if "gn_glu_fwd" in r["Name"]:
        print("fpb", sys.argv[2], "gn_glu_fwd avg us", round(float(r["AverageNs"]) / 1e3, 2), "ms/step", d["ms_per_step"])
PY
done
