import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for p in [f"{d}/p1/run_counter_collection.csv", f"{d}/p2/run_counter_collection.csv"]:
    for r in csv.DictReader(open(p)):
        k = (r["Kernel_Name"].split("(")[0][-45:], r["Grid_Size"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    n = len(cnt[k]) / 1.0
    m = v["SQ_INSTS_MFMA"] / n
    if not m:
        continue
    wc = v["SQ_WAVE_CYCLES"]
    print(f"{k[0]:45s} grid={k[1]:>7s} mfma_busy={v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f} "
          f"valu/mfma={v['SQ_INSTS_VALU'] / v['SQ_INSTS_MFMA']:.2f} salu/mfma={v['SQ_INSTS_SALU'] / v['SQ_INSTS_MFMA']:.2f} "
          f"lds/mfma={v['SQ_INSTS_LDS'] / v['SQ_INSTS_MFMA']:.2f} wait_any={v['SQ_WAIT_ANY'] / wc:.2f} "
          f"wait_inst={v['SQ_WAIT_INST_ANY'] / wc:.2f} wait_lds={v['SQ_WAIT_INST_LDS'] / wc:.2f} active={v['SQ_ACTIVE_INST_ANY'] / wc:.2f} "
          f"lds_conf={v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
