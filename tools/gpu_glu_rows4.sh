#!/bin/bash
# GN-GLU forward with four rows' loads in flight (build -D VQX_GLU_ROWS4=1 ->
# lib/libvqx_r4.so) vs the default two: GN/GLU tests on the variant, then
# per-kernel times from alternating rocprofv3 --stats runs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/glu4
mkdir -p $O
VQX_LIB=vae_npvc_amd/lib/libvqx_r4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_step.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "glu or gn or step" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in base r4 base r4; do
  L=vae_npvc_amd/lib/libvqx.so; [ $v = r4 ] && L=vae_npvc_amd/lib/libvqx_r4.so
  VQX_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p$v -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --fp32-steps 0 --vq-reps 0 --no-probe --steps 20 --warmup 5 > $O/b$v.json 2> $O/b$v.err || exit $?
  python3 - $O/p$v/run_kernel_stats.csv $v $O/b$v.json <<'PY'
import csv, json, sys
d = json.load(open(sys.argv[3]))
for r in csv.DictReader(open(sys.argv[1])):
    if "gn_glu_fwd" in r["Name"]:
        print(sys.argv[2], "gn_glu_fwd avg us", round(float(r["AverageNs"]) / 1e3, 2), "ms/step", d["ms_per_step"])
PY
done
