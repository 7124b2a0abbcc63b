"""Per-round plan/accept durations of one solve (default: the last) in a rocprofv3 kernel
trace (tools/gpu_trace.sh): python tools/trace_rounds.py <kernel_trace.csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
which = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "--all" else -1  # solve index (k_reset_units)
end = starts[which + 1] if which != -1 and which + 1 < len(starts) else len(rows)
seq = rows[starts[which]:end]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rs = [i for i, r in enumerate(seq) if ("k_round_start" in r["Kernel_Name"] or "k_round_begin" in r["Kernel_Name"])]
span = (max(int(r["End_Timestamp"]) for r in seq) - int(seq[0]["Start_Timestamp"])) / 1e3
tot = {}
for r in seq:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kp::(anonymous namespace)::", "")[:40]
    tot[n] = tot.get(n, 0) + dur(r)
print(f"rounds {len(rs)} span {span:.0f} us")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {v:9.0f} us  {n}")
for ri, a in enumerate(rs):
    b = rs[ri + 1] if ri + 1 < len(rs) else len(seq)
    acc = [dur(r) for r in seq[a:b] if "k_accept" in r["Kernel_Name"]]
    pl = [dur(r) for r in seq[a:b] if "k_plan" in r["Kernel_Name"]]
    if ri < 6 or ri % 10 == 0 or ri > len(rs) - 3:
        print(ri, "acc", " ".join("%.0f" % x for x in acc), "| plan", " ".join("%.0f" % x for x in pl))
if "--all" in sys.argv:
    print("round: plan_sum accept_sum other_sum (us)")
    for ri, a in enumerate(rs):
        b = rs[ri + 1] if ri + 1 < len(rs) else len(seq)
        acc = sum(dur(r) for r in seq[a:b] if "k_accept" in r["Kernel_Name"])
        pl = sum(dur(r) for r in seq[a:b] if "k_plan" in r["Kernel_Name"])
        ot = sum(dur(r) for r in seq[a:b]) - acc - pl
        print(f"{ri}:{pl:.0f}/{acc:.0f}/{ot:.0f}", end=" ")
    print()
