# L2 hit/miss and fabric read requests per kernel of two bench steps (one --pmc pass, no trace domains).
# usage: bash tools/gpu_pmc_l2.sh TAG
TAG=${1:-x}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$TAG/pmc_l2
mkdir -p $O
P="python3 bench.py --steps 2 --warmup 1 --no-probe --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/p -o run --output-format csv -- $P > $O/p.log 2>&1 || exit $?
python3 - $O <<'PY'
import csv, collections, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(f"{d}/p/run_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0][-44:]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
rows = sorted(agg.items(), key=lambda kv: -kv[1]["TCC_EA0_RDREQ_sum"])
with open(f"{d}/summary.txt", "w") as f:
    for k, v in rows[:20]:
        c = len(n[k]); h, m = v["TCC_HIT_sum"], v["TCC_MISS_sum"]
        line = (f"{k:44s} disp={c:3d} L2 hit={h / max(h + m, 1):.2f} req/disp={(h + m) / c / 1e6:.2f}M "
                f"ea_rd/disp={v['TCC_EA0_RDREQ_sum'] / c / 1e6:.2f}M ea_wr/disp={v['TCC_EA0_WRREQ_sum'] / c / 1e6:.2f}M")
        print(line); f.write(line + "\n")
PY
