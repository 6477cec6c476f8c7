"""Per-kernel SQ counter summary for kernels with or without MFMAs (the
non-GEMM kernels): instructions per wave by class and where the waves wait.
usage: python tools/pmc_any.py gpurun_out/TAG/pmc [name-filter]"""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for p in [f"{d}/p1/run_counter_collection.csv", f"{d}/p2/run_counter_collection.csv"]:
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"].split("(")[0][-45:]
        if flt not in name:
            continue
        k = (name, r["Grid_Size"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
for k, v in sorted(agg.items()):
    n = max(len(cnt[k]), 1)
    waves = max(v["SQ_WAVES"], 1)
    wc = max(v["SQ_WAVE_CYCLES"], 1)
    print(f"{k[0]:45s} grid={k[1]:>8s} launches={n} waves/launch={waves / n:.0f} "
          f"valu/wave={v['SQ_INSTS_VALU'] / waves:.0f} lds/wave={v['SQ_INSTS_LDS'] / waves:.0f} "
          f"salu/wave={v['SQ_INSTS_SALU'] / waves:.0f} wave_cycles/wave={wc / waves:.0f} "
          f"wait_any={v['SQ_WAIT_ANY'] / wc:.2f} wait_inst={v['SQ_WAIT_INST_ANY'] / wc:.2f} "
          f"wait_lds={v['SQ_WAIT_INST_LDS'] / wc:.2f} active={v['SQ_ACTIVE_INST_ANY'] / wc:.2f} "
          f"busy_cycles/launch={v['SQ_BUSY_CYCLES'] / n:.0f} gui_active/launch={v['GRBM_GUI_ACTIVE'] / n:.0f}")
