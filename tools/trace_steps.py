"""Per-kernel time per bf16 training step from a rocprofv3 kernel trace of bench.py:
steps are the windows between consecutive adam_kernel / adam_wn_kernel launches; windows holding
fp32 GEMMs (the bench's fp32 leg) or more than one step's launches are skipped.
python tools/trace_steps.py TRACE_CSV [TOP]"""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
ad = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("vqx::adam_kernel", "vqx::adam_wn_kernel"))]
wins = []
for a, b in zip(ad[:-1], ad[1:]):
    seg = rows[a:b]
    if any(re.search(r"(conv|dual|wgrad)\w*<float", r["Kernel_Name"]) for r in seg):  # fp32 GEMMs
        continue
    wins.append(seg)
n = {len(w) for w in wins}
common = max(n, key=lambda k: sum(len(w) == k for w in wins))
wins = [w for w in wins if len(w) == common]
tot, cnt = defaultdict(float), defaultdict(int)
span = busy = 0.0
for w in wins:
    t0 = int(w[0]["Start_Timestamp"])
    last = t0
    for r in w:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        tot[name] += (e - s) / 1e3
        cnt[name] += 1
        s = max(s, last)
        if e > s:
            busy += (e - s) / 1e3
            last = e
    span += (int(w[-1]["End_Timestamp"]) - t0) / 1e3
k = len(wins)
print(f"{k} bf16 steps of {common} launches: kernel time {sum(tot.values()) / k / 1e3:.3f} ms/step, "
      f"GPU busy {busy / k / 1e3:.3f} of {span / k / 1e3:.3f} ms span")
for name, t in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{t / k / 1e3:7.3f} ms {cnt[name] // k:4d}x avg {t / cnt[name]:7.1f} us  {name[:100]}")
