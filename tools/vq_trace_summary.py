"""Median per-kernel durations of tools/vq_bench.py from a rocprofv3 kernel trace (us)."""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/vqprof/vq_kernel_trace.csv")))
seq = sorted((int(r["Start_Timestamp"]), r["Kernel_Name"].split("(")[0], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
             for r in rows)
seq = [x for x in seq if "vqx" in x[1]]
i = 0
for cfg in ["K128 randn", "K128 rows", "K512 randn", "K512 rows", "K1024 randn", "K1024 rows"]:
    full, nost, only = seq[i:i + 23 * 4], seq[i + 23 * 4:i + 23 * 6], seq[i + 23 * 6:i + 23 * 7]
    i += 23 * 7

    def med(lst, name):
        v = [x[2] for x in lst if name in x[1]]
        return statistics.median(v) if v else 0.0
    print(f"{cfg:12s} forward {med(full, 'vq_forward'):6.1f} (idx-only {med(only, 'vq_forward'):6.1f})  "
          f"sum {med(full, 'sum_partials'):5.1f}  stats {med(full, 'vq_stats_kernel'):5.1f}  "
          f"reduce {med(full, 'reduce'):5.1f}")
