"""Summary of a rocprofv3 --rccl-trace run (tools/gpu_r06b.sh: the one-rank
RCCL solves of tests/test_gpu_rccl.py): the RCCL API stats, and per
communicator lifetime (ncclCommInitRank .. ncclCommDestroy) the number of
ncclAllGather calls and the solves' k_reset_units launches in it.
python tools/rccl_summary.py <dir with run_rccl_api_trace.csv, run_rccl_api_stats.csv, run_kernel_trace.csv>"""
import csv
import os
import sys

d = sys.argv[1]
api = sorted(csv.DictReader(open(os.path.join(d, "run_rccl_api_trace.csv"))),
             key=lambda r: int(r["Start_Timestamp"]))
ker = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
print("# RCCL API stats (rocprofv3 --rccl-trace --stats)")
print(open(os.path.join(d, "run_rccl_api_stats.csv")).read().strip())
print()
print("# per communicator: ncclAllGather calls and solves (k_reset_units launches) while it lived")
lives, cur = [], None
for r in api:
    if r["Function"] == "ncclCommInitRank":
        cur = {"t0": int(r["Start_Timestamp"]), "ag": [], "t1": None}
    elif r["Function"] == "ncclAllGather" and cur is not None:
        cur["ag"].append(int(r["Start_Timestamp"]))
    elif r["Function"] == "ncclCommDestroy" and cur is not None:
        cur["t1"] = int(r["End_Timestamp"])
        lives.append(cur)
        cur = None
for i, L in enumerate(lives):
    solves = sorted(int(k["Start_Timestamp"]) for k in ker if "k_reset_units" in k["Kernel_Name"]
                    and L["t0"] <= int(k["Start_Timestamp"]) <= L["t1"])
    per = []
    for j, s in enumerate(solves):
        e = solves[j + 1] if j + 1 < len(solves) else L["t1"]
        per.append(sum(1 for t in L["ag"] if s <= t < e))
    print(f"communicator {i}: {len(L['ag'])} ncclAllGather calls; solves {len(solves)}; "
          f"all-gathers from each solve start to the next: {per}")
names = {}
for k in ker:
    n = k["Kernel_Name"]
    if "nccl" in n.lower() or "rccl" in n.lower():
        names[n[:80]] = names.get(n[:80], 0) + 1
print("RCCL device kernels in the kernel trace:", names if names else "none (a one-rank all-gather is a device copy)")
