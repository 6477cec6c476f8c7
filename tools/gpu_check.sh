#!/bin/bash
# Fused-launch tests, the whole GPU suite, then the default bench line (dominant-kernel probe) beside a --no-probe run.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/check
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "fused_dgrad_wgrad" > $O/tests_fused.log 2>&1 || { tail -40 $O/tests_fused.log; exit 1; }
tail -1 $O/tests_fused.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests_all.log 2>&1 || { tail -40 $O/tests_all.log; exit 1; }
tail -1 $O/tests_all.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --fp32-steps 0 > $O/bench_probe$i.json 2> $O/bench_probe$i.err || exit $?
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --no-probe > $O/bench_noprobe$i.json 2> $O/bench_noprobe$i.err || exit $?
done
python3 - <<'PY'
import json
for n in ("probe1", "noprobe1", "probe2", "noprobe2"):
    d = json.load(open(f"gpurun_out/check/bench_{n}.json"))
    r = d["roofline"] or {}
    print(n, d["ms_per_step"], d["value"], r.get("kernel"), r.get("frac"), r.get("avg_launch_us"), r.get("launches_per_step"),
          (d.get("vq") or {}).get("us"))
PY
