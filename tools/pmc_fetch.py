"""Per-launch FETCH_SIZE (x2, the gfx950 correction) / WRITE_SIZE of k_score_topk in a
rocprofv3 --pmc counter_collection.csv: python tools/pmc_fetch.py <csv>"""
import collections
import csv
import sys

per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "k_score_topk" in r["Kernel_Name"]:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = [d[c] for d in per.values() if c in d]
    if v:
        mul = 2.0 if c == "FETCH_SIZE" else 1.0
        print(f"k_score_topk {c}: {len(v)} launches, {mul * 1024 * sum(v) / len(v) / 1e6:.3f} MB per launch "
              f"(round 0: {mul * 1024 * v[0] / 1e6:.3f} MB)")
