"""Per-round view of a rocprofv3 kernel trace of bench.py: kernel durations
and the gaps between consecutive kernels, for the last solve in the trace."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.replace("kp::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:28]
# split into solves at k_reset_units
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
lo = starts[-1]
hi = len(rows)
seq = rows[lo:hi]
t0 = int(seq[0]["Start_Timestamp"])
tend = int(seq[-1]["End_Timestamp"])
print(f"last solve: {len(seq)} kernels, span {(tend - t0) / 1e3:.1f} us")
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seq)
print(f"busy {busy / 1e3:.1f} us, gaps {(tend - t0 - busy) / 1e3:.1f} us")
agg = {}
prev_end = None
for r in seq:
    n = short(r["Kernel_Name"])
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    g = int(r["Start_Timestamp"]) - prev_end if prev_end else 0
    a = agg.setdefault(n, [0, 0, 0])
    a[0] += 1
    a[1] += d
    a[2] += g
    prev_end = int(r["End_Timestamp"])
for n, (c, d, g) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{c:6d} x {n:30s} busy {d / 1e3:9.1f} us  gaps-before {g / 1e3:8.1f} us")
if len(sys.argv) > 2:
    rnd = int(sys.argv[2])
    # print the kernels of round `rnd` (rounds start at k_flag_active)
    rs = [i for i, r in enumerate(seq) if "k_flag_active" in r["Kernel_Name"]]
    a, b = rs[rnd], rs[rnd + 1] if rnd + 1 < len(rs) else len(seq)
    for r in seq[a:b]:
        print(f"  {short(r['Kernel_Name']):30s} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.2f} us grid {r['Grid_Size_X']}")
