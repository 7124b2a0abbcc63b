"""Per-kernel totals of the second solve in a rocprofv3 kernel trace
(tools/gpu_trace.sh), plus the first launches of chosen kernels."""
import collections
import csv
import re
import sys

path = sys.argv[1]
show = sys.argv[2].split(",") if len(sys.argv) > 2 else ["k_score_topk", "k_merge_topk", "k_score32", "k_select_t"]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[starts[1]:starts[2] if len(starts) > 2 else len(rows)]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seq:
    m = re.search(r"(k_\w+|rocprim|__amd\w+)", r["Kernel_Name"])
    n = m.group(0) if m else r["Kernel_Name"][:40]
    agg[n][0] += 1
    agg[n][1] += dur(r)
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print("solve span %.0f us, kernel sum %.0f us" % (span, sum(v[1] for v in agg.values())))
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
    print("%8.0f us %5d  %s" % (t, c, n))
for k in show:
    d = [dur(r) for r in seq if k in r["Kernel_Name"]]
    if d:
        print(k, "first:", " ".join("%.0f" % x for x in d[:10]), "| last:", " ".join("%.0f" % x for x in d[-5:]))
