# bwd_streams: bit-identity tests, same-box A/B and the step trace of both schedules
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/bs2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_step.py -k "concurrent or fused" > gpurun_out/bs2/t.log 2>&1 || { tail -5 gpurun_out/bs2/t.log; exit 1; }
tail -1 gpurun_out/bs2/t.log
bash tools/gpu_ab_engine.sh bs2/ab '{"bwd_streams":false}' || exit 1
bash tools/gpu_prof_step.sh bs2/pc > /dev/null || exit 1
VQX_ENGINE='{"bwd_streams":false}' bash tools/gpu_prof_step.sh bs2/ps > /dev/null || exit 1
for t in pc ps; do echo "$t $(python3 tools/trace_steps.py gpurun_out/bs2/$t/prof/run_kernel_trace.csv 60 | grep -E 'kernel time|dual_tr|dual_k1_3|conv_pp|gn_bwd' | sed 's/  */ /g' | tr '\n' '|')"; done
