#!/bin/bash
# Fused DGRAD+WGRAD launches (vqx_gemm_dual.hip): bit-identity tests, the whole GPU suite, same-box A/B of VQX_DUAL, probe.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/dual
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "fused_dgrad_wgrad" > gpurun_out/dual/tests_fused.log 2>&1 || { tail -40 gpurun_out/dual/tests_fused.log; exit 1; }
tail -2 gpurun_out/dual/tests_fused.log
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/dual/tests_all.log 2>&1 || { tail -40 gpurun_out/dual/tests_all.log; exit 1; }
  tail -2 gpurun_out/dual/tests_all.log
fi
bash tools/gpu_ab_env.sh dual VQX_DUAL ${AB_A:-0} ${AB_B:-1} || exit $?
VQX_BENCH_KERNELS=2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --fp32-steps 0 \
  > gpurun_out/dual/bench_k.json 2> gpurun_out/dual/bench_k.err || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/dual/bench_k.json"))
print(d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["avg_launch_us"])
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["seconds"])[:8]:
    print(round(v["seconds"] * 1e3 / 4, 3), "ms/step", v["launches"] // 4, round(v["avg_us"], 1), round(v["tflops"], 1), k)
for k, v in sorted(d["layers"].items(), key=lambda kv: -kv[1][0] * kv[1][1])[:16]:
    print(v, k)
PY
