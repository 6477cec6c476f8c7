# GN-GLU forward A/B: the in-tree library (whole GPU suite first) vs a variant
# built into lib/libvqx_r4.so (build.py -D ... --out; rounds so far: four rows
# in flight, then the unfused tanh*sigmoid as the baseline), per-kernel times
# from alternating rocprofv3 --stats runs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/glu4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
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
