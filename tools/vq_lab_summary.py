"""Median vq_forward_kernel duration per K for each VQX_VQ_LAB variant (tools/vq_lab.sh output)."""
import csv
import glob
import statistics

for v in range(4):
    f = glob.glob(f"gpurun_out/vqlab/v{v}/**/*kernel_trace.csv", recursive=True)
    if not f:
        continue
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "vq_forward" in r["Kernel_Name"]]
    per = [d[i * 53:(i + 1) * 53] for i in range(len(d) // 53)]
    print(f"LAB={v}: " + "  ".join(f"K{k}={statistics.median(p):.2f}" for k, p in zip((16, 64, 128, 256, 512, 1024, 2048), per)))
