"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel ms/step.
python tools/prof_summary.py DIR STEPS"""
import csv
import sys

d, steps = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time per step: {tot / 1e6 / steps:.3f} ms")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.3f} ms {int(r['Calls']) // steps:4d}x avg "
          f"{float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:110]}")
