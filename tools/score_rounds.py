"""Per-round filter+score / select durations of the last solve in a rocprofv3
kernel trace (rows of round r = the active count, read from the next round's
select grid bound)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[st[-1]:]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
Ns = (N + 63) // 64 * 64
out, sc = [], None
for r in seq:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_score32" in n or "k_score<" in n:
        sc = d
    if "k_select" in n:
        out.append([int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), sc, d])
tot_b = tot_s = tot_sel = 0
for i, (bound, s, sel) in enumerate(out):
    act = out[i + 1][0] if i + 1 < len(out) else bound
    act = min(act, bound)
    b = act * Ns * 4
    tot_b += b
    tot_s += s
    tot_sel += sel
    if i < 14 or i % 8 == 0:
        print(f"round {i:2d} rows {act:6d} score {s:7.1f} us {b / s / 1e3:6.0f} GB/s  select {sel:7.1f} us {b / sel / 1e3:6.0f} GB/s")
print(f"total: score {tot_s:.0f} us ({tot_b / tot_s / 1e3:.0f} GB/s), select {tot_sel:.0f} us ({tot_b / tot_sel / 1e3:.0f} GB/s), {tot_b / 1e9:.2f} GB")
