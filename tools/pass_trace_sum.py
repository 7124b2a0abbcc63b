"""Per-pass plan / accept durations of the last solve in a rocprofv3 kernel
trace: python tools/pass_trace_sum.py <kernel_trace.csv>. Prints, by pass
index, the summed and maximum accept and plan time over the solve's rounds,
and the rounds whose passes cost most (a round starts at k_round_begin)."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
rb = [i for i, r in enumerate(seq) if "k_round_begin" in r["Kernel_Name"] or "k_round_start" in r["Kernel_Name"]]
acc_p, plan_p = defaultdict(list), defaultdict(list)
per_round = []
for ri, a in enumerate(rb):
    b = rb[ri + 1] if ri + 1 < len(rb) else len(seq)
    acc = [dur(r) for r in seq[a:b] if "k_accept" in r["Kernel_Name"]]
    pl = [dur(r) for r in seq[a:b] if "k_plan" in r["Kernel_Name"]]
    for p, x in enumerate(acc):
        acc_p[p].append(x)
    for p, x in enumerate(pl):
        plan_p[p].append(x)
    per_round.append((ri, sum(acc), sum(pl), acc, pl))
print(f"rounds {len(rb)}; accept total {sum(x[1] for x in per_round):.0f} us, plan total {sum(x[2] for x in per_round):.0f} us")
print("pass: accept sum/max us | plan sum/max us")
for p in sorted(acc_p):
    print(f"{p:3d}: {sum(acc_p[p]):9.0f} {max(acc_p[p]):7.1f} | {sum(plan_p[p]):9.0f} {max(plan_p[p]):7.1f}")
print("most expensive rounds (accept us per pass):")
for ri, sa, sp, acc, pl in sorted(per_round, key=lambda x: -x[1])[:8]:
    print(f"round {ri}: accept {sa:.0f} plan {sp:.0f} | " + " ".join(f"{x:.0f}" for x in acc))
