"""Per-launch durations of k_pass_loop (and the per-pass kernels) of the
second solve in a rocprofv3 kernel trace: python tools/loop_trace.py run_kernel_trace.csv"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[starts[1]:starts[2] if len(starts) > 2 else len(rows)]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rnd, out = -1, []
for r in seq:
    n = r["Kernel_Name"]
    if "k_round_begin" in n or "k_round_start" in n:
        rnd += 1
    m = re.search(r"(k_\w+)", n)
    k = m.group(0) if m else n[:30]
    out.append((rnd, k, dur(r), r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", "")))
tot = {}
for rnd_, k, d, g, wg in out:
    tot.setdefault(rnd_, {}).setdefault(k, [0, 0.0])
    tot[rnd_][k][0] += 1
    tot[rnd_][k][1] += d
for rnd_ in sorted(tot):
    print(rnd_, " ".join(f"{k}:{c}x{t:.0f}" for k, (c, t) in sorted(tot[rnd_].items())))
