"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_pmc.sh into
profiles/<round>_pmc.json: per-launch HBM-side bytes of the filter+score and
select kernels of one config-#3 solve. Units follow MI355X_MICROARCH.md: the
counters are in KB; FETCH_SIZE reports half of a 16-B-per-lane streaming read
on gfx950 and is doubled; WRITE_SIZE is exact for 16-B-per-lane stores."""
import csv
import json
import sys
from collections import defaultdict

src, out = sys.argv[1], sys.argv[2]
res = defaultdict(lambda: defaultdict(list))
for C in ("FETCH_SIZE", "WRITE_SIZE"):
    for r in csv.DictReader(open(f"{src}/{C}/run_counter_collection.csv")):
        n = r["Kernel_Name"].replace("kp::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        res[n][C].append(float(r["Counter_Value"]))
summary = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                     "bench.py --steps 1 --warmup 0 (config #3)",
           "fetch_correction": 2.0, "kernels": {}}
for n, d in res.items():
    f, w = d.get("FETCH_SIZE", []), d.get("WRITE_SIZE", [])
    launches = max(len(f), len(w))
    fetch_b = 2.0 * 1024 * sum(f) / max(len(f), 1)
    write_b = 1024 * sum(w) / max(len(w), 1)
    summary["kernels"][n] = {"launches_per_solve": launches,
                             "fetch_bytes_per_launch": fetch_b,
                             "write_bytes_per_launch": write_b,
                             "traffic_bytes_per_launch": fetch_b + write_b,
                             "max_launch_write_bytes": 1024 * max(w) if w else 0.0}
json.dump(summary, open(out, "w"), indent=1)
print(json.dumps(summary, indent=1))
