"""Print a rocprofv3 kernel_stats.csv as a short table (per-solve numbers
when --solves is given)."""
import csv
import sys

path = sys.argv[1]
solves = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / solves:.3f} ms per solve")
for r in rows[:25]:
    n = r["Name"]
    n = n.replace("kp::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    print(f"{int(r['Calls']) / solves:8.1f} calls {float(r['TotalDurationNs']) / 1e6 / solves:8.3f} ms "
          f"avg {float(r['AverageNs']) / 1e3:7.2f} us max {float(r['MaxNs']) / 1e3:7.1f} us  {n}")
