"""HBM traffic per dispatch from two rocprofv3 --pmc passes (FETCH_SIZE, then
WRITE_SIZE) over `bench.py --no-probe`, with the MI355X_MICROARCH.md gfx950
corrections: FETCH_SIZE counts half the bytes of a wide coalesced read
(double it); WRITE_SIZE is exact for 16-B stores.  rocprofv3 reports both in
KiB.  Unit check: adam_kernel moves 4 reads + 3 writes of the flat fp32
parameter vector, a known byte count printed next to the measurement.

python tools/pmc_hbm.py DIR N_PARAMS OUT.json"""
import collections
import csv
import json
import sys

d, n_params, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
per = collections.defaultdict(lambda: collections.defaultdict(float))  # (dispatch) -> counter -> value
name = {}
for sub, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
        if r["Counter_Name"] != ctr:
            continue
        key = (sub, r["Dispatch_Id"])
        per[key][ctr] += float(r["Counter_Value"])
        name[key] = r["Kernel_Name"].split("(")[0].replace("void ", "")

agg = collections.defaultdict(lambda: {"fetch_bytes": [], "write_bytes": []})
for (sub, _), v in per.items():
    k = name[(sub, _)]
    if sub == "fetch":
        agg[k]["fetch_bytes"].append(2.0 * v["FETCH_SIZE"] * 1024)  # x2: gfx950 half-count of wide reads
    else:
        agg[k]["write_bytes"].append(v["WRITE_SIZE"] * 1024)
res = {}
for k, v in agg.items():
    f, w = v["fetch_bytes"], v["write_bytes"]
    if not f or not w:
        continue
    res[k] = {"dispatches": len(f), "read_bytes_per_launch": sum(f) / len(f), "write_bytes_per_launch": sum(w) / len(w),
              "hbm_bytes_per_launch": sum(f) / len(f) + sum(w) / len(w)}
adam = res.get("vqx::adam_kernel") or res.get("vqx::adam_wn_kernel")
calib = None
if adam:
    # adam_wn_kernel (round 5) also writes the Conv1d packed weights (2 B per weight in bf16)
    # and the row norms: its reads are the same 16 B per parameter, its writes 12 B + those
    calib = {"kernel": "vqx::adam_kernel" if "vqx::adam_kernel" in res else "vqx::adam_wn_kernel",
             "adam_expected_read": 16.0 * n_params, "adam_expected_write_min": 12.0 * n_params,
             "adam_measured_read": adam["read_bytes_per_launch"], "adam_measured_write": adam["write_bytes_per_launch"]}
json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py --no-probe",
           "correction": "read = 2 x FETCH_SIZE (gfx950 wide-read half count); KiB -> bytes",
           "calibration": calib, "kernels": res}, open(out, "w"), indent=1)
for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches"])[:15]:
    print(f"{v['dispatches']:4d}x {v['read_bytes_per_launch'] / 1e6:9.2f} MB rd {v['write_bytes_per_launch'] / 1e6:9.2f} MB wr  {k}")
print("calibration", calib)
