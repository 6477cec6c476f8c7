#!/bin/bash
# Wide tap-reuse weight gradient (wgrad_tr2_kernel): parity tests, same-box A/B of VQX_WGRAD_WIDE, per-layer probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wide
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "wgrad" > gpurun_out/wide/tests.log 2>&1 || { tail -30 gpurun_out/wide/tests.log; exit 1; }
tail -2 gpurun_out/wide/tests.log
bash tools/gpu_ab_env.sh wide VQX_WGRAD_WIDE 0 1 || exit $?
VQX_WGRAD_WIDE=1 VQX_BENCH_KERNELS=2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --fp32-steps 0 \
  > gpurun_out/wide/bench_k.json 2> gpurun_out/wide/bench_k.err || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/wide/bench_k.json"))
print(d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d["vq"])
for k, v in sorted(d["layers"].items(), key=lambda kv: -kv[1][0] * kv[1][1])[:12]:
    print(v, k)
PY
