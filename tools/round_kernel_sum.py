"""Per-round durations of the per-round kernels in the last solve of a
rocprofv3 kernel trace: python tools/round_kernel_sum.py <kernel_trace.csv>
(a round starts at k_round_begin / k_round_start; prints every 10th round and
the totals)."""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
name = lambda r: (re.search(r"(k_\w+)", r["Kernel_Name"]) or re.search(r"(.{0,30})", r["Kernel_Name"])).group(1)
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rb = [i for i, r in enumerate(seq) if re.search(r"k_round_(begin|start)", r["Kernel_Name"])]
tot = defaultdict(float)
per = []
for ri, a in enumerate(rb):
    b = rb[ri + 1] if ri + 1 < len(rb) else len(seq)
    d = defaultdict(float)
    for r in seq[a:b]:
        d[name(r)] += dur(r)
    per.append(d)
    for k, v in d.items():
        tot[k] += v
keys = [k for k, _ in sorted(tot.items(), key=lambda x: -x[1]) if k not in ("k_plan", "k_accept")][:8]
print("round " + " ".join(f"{k[:14]:>14}" for k in keys))
for ri, d in enumerate(per):
    if ri % 10 == 0 or ri < 3:
        print(f"{ri:5d} " + " ".join(f"{d.get(k, 0):14.1f}" for k in keys))
print("total " + " ".join(f"{tot[k]:14.1f}" for k in keys))
