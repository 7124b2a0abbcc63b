"""Per-round pass cost of the last solve in a rocprofv3 kernel trace:
python tools/c3_round_passes.py <kernel_trace.csv>

For every round (delimited by k_round_begin / k_round_start): the number of
k_plan / k_accept launches, their summed and largest durations (us), the
k_plan grid (workgroups: the round's slot bound) and the other kernels' time.
Then cumulative shares by round size, to see where the pass loop's time is."""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
name = lambda r: (re.search(r"(k_\w+)", r["Kernel_Name"]) or re.search(r"(.{0,30})", r["Kernel_Name"])).group(1)
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
grid = lambda r: int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
wg = lambda r: max(1, int(r.get("Workgroup_Size", r.get("Workgroup_Size_X", 1)) or 1))
rb = [i for i, r in enumerate(seq) if re.search(r"k_round_(begin|start)", r["Kernel_Name"])]
out = []
for ri, a in enumerate(rb):
    b = rb[ri + 1] if ri + 1 < len(rb) else len(seq)
    d = defaultdict(float)
    n = defaultdict(int)
    mx = defaultdict(float)
    pg = 0
    for r in seq[a:b]:
        k = name(r)
        d[k] += dur(r)
        n[k] += 1
        mx[k] = max(mx[k], dur(r))
        if k == "k_plan" and not pg:
            pg = grid(r) // wg(r)
    other = sum(v for k, v in d.items() if k not in ("k_plan", "k_accept"))
    out.append((ri, n["k_plan"], d["k_plan"], mx["k_plan"], d["k_accept"], mx["k_accept"], pg, other))
print("round passes  plan_us  plan_max  acc_us  acc_max  plan_wgs  other_us")
for t in out:
    print(f"{t[0]:5d} {t[1]:6d} {t[2]:8.1f} {t[3]:8.1f} {t[4]:7.1f} {t[5]:8.1f} {t[6]:9d} {t[7]:9.1f}")
tp = sum(t[2] for t in out)
ta = sum(t[4] for t in out)
to = sum(t[7] for t in out)
npass = sum(t[1] for t in out)
print(f"total passes {npass} plan {tp:.1f} accept {ta:.1f} other {to:.1f} us")
for lim in (16, 64, 256, 1024, 4096):
    sel = [t for t in out if t[6] <= lim]
    print(f"rounds with plan grid <= {lim:5d} wgs: {len(sel):3d} rounds, {sum(t[1] for t in sel):4d} passes, "
          f"plan {sum(t[2] for t in sel):8.1f} + accept {sum(t[4] for t in sel):8.1f} us")
