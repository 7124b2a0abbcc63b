"""Summarise gpurun_out/evidence (tools/gpu_evidence.sh) into profiles/<round>_*.

usage: python tools/evidence_summary.py r02 [gpurun_out/evidence [out_dir]]
(out_dir defaults to profiles/; tools/gpu_evidence.sh summarises on the GPU
box into gpurun_out/evidence/summary and drops the raw traces)

Units follow MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are in KB;
FETCH_SIZE reports half of a 16-B-per-lane streaming read on gfx950 and is
doubled; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles.
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

rnd = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/evidence"
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = sys.argv[3] if len(sys.argv) > 3 else os.path.join(repo, "profiles")
os.makedirs(prof, exist_ok=True)


def kname(s):
    m = re.search(r"(k_\w+|rocprim|__amd\w+)", s)
    return m.group(0) if m else s[:40]


def copy(rel, dst):
    p = os.path.join(src, rel)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(prof, f"{rnd}_{dst}"))
        return True
    return False


copy("pytest_gpu.log", "pytest_gpu.log")
copy("bench.json", "bench.json")
copy("prof/run_kernel_stats.csv", "kernel_stats.csv")
copy("prof/bench_prof.json", "bench_profiled_cmd.json")
copy("profsm/run_kernel_stats.csv", "kernel_stats_score_matrix.csv")
copy("profsm/score_dev.log", "score_dev_profiled.txt")
copy("prof45/run_kernel_stats.csv", "kernel_stats_config4_config5.csv")
copy("prof45/bench_prof.json", "bench_profiled_config4_config5.json")


# per-solve kernel totals of the profiled config #3 steps (warmup 1 + steps 3)
def per_solve(trace, solves, out):
    if not os.path.exists(trace):
        return
    rows = list(csv.DictReader(open(trace)))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        n = kname(r["Kernel_Name"])
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values())
    with open(out, "w") as f:
        f.write(f"# {trace}: kernel totals / {solves} solves (us per solve, launches per solve)\n")
        f.write(f"# all kernels: {tot / solves:.0f} us per solve\n")
        for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
            f.write(f"{t / solves:10.1f} us {c / solves:8.1f}  avg {t / max(c, 1):8.2f} us  {n}\n")


per_solve(os.path.join(src, "prof/run_kernel_trace.csv"), 4,
          os.path.join(prof, f"{rnd}_kernel_stats_per_solve.txt"))

# PMC: per kernel, per-launch HBM bytes and the SQ counters of one solve
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for grp in ("FETCH_SIZE", "WRITE_SIZE", "SQ1", "LDS"):
    p = os.path.join(src, "pmc", grp, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(p)):
        per[(kname(r["Kernel_Name"]), int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
    for (n, _), d in per.items():
        for c, v in d.items():
            pmc[n][c].append(v)

bench = {}
bp = os.path.join(src, "prof", "bench_prof.json")
if os.path.exists(bp):
    bench = json.load(open(bp))
pairs = bench.get("config", {}).get("pairs_scored")

hbm = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --steps 1 "
                 "--warmup 0 (config #3, one solve)", "fetch_correction": 2.0, "kernels": {}}
valu = {"source": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES "
                  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY (one pass), one config #3 solve",
        "pairs_scored_per_solve": pairs, "kernels": {}}
lds = {"source": "rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES",
       "kernels": {}}
for n, d in pmc.items():
    f, w = d.get("FETCH_SIZE", []), d.get("WRITE_SIZE", [])
    if f or w:
        fb = 2.0 * 1024 * sum(f) / max(len(f), 1)
        wb = 1024 * sum(w) / max(len(w), 1)
        hbm["kernels"][n] = {"launches_per_solve": max(len(f), len(w)),
                             "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                             "traffic_bytes_per_launch": fb + wb}
    if "SQ_INSTS_VALU" in d:
        s = {c: sum(v) for c, v in d.items() if c.startswith("SQ_") and c not in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE")}
        e = {"launches_per_solve": len(d["SQ_INSTS_VALU"]), "per_solve": s}
        wc = s.get("SQ_WAVE_CYCLES", 0)
        if wc:
            e["wave_cycle_split"] = {"wait_any": s.get("SQ_WAIT_ANY", 0) / wc,
                                     "wait_inst_any": s.get("SQ_WAIT_INST_ANY", 0) / wc,
                                     "active_inst_any": s.get("SQ_ACTIVE_INST_ANY", 0) / wc}
        if s.get("SQ_WAVES"):
            e["valu_insts_per_wave"] = s["SQ_INSTS_VALU"] / s["SQ_WAVES"]
        if pairs and n in ("k_score_topk", "k_score32", "k_select_t", "k_merge_topk"):
            e["valu_lane_ops_per_pair"] = 64.0 * s["SQ_INSTS_VALU"] / pairs
        valu["kernels"][n] = e
    if "SQ_LDS_BANK_CONFLICT" in d:
        bc, act = sum(d["SQ_LDS_BANK_CONFLICT"]), sum(d.get("SQ_LDS_IDX_ACTIVE", [0]))
        lds["kernels"][n] = {"bank_conflict_cycles": bc, "lds_active_cycles": act,
                             "conflict_frac": bc / act if act else None,
                             "lds_insts": sum(d.get("SQ_INSTS_LDS", [0]))}
# score + threshold stages alone (the no-select build, round 0 only): the
# select phase's VALU / SALU per pair is the full kernel's minus these
ns = os.path.join(src, "pmc", "SQ_NOSEL", "run_counter_collection.csv")
if os.path.exists(ns) and "k_score_topk" in valu["kernels"]:
    tot = collections.defaultdict(float)
    for r in csv.DictReader(open(ns)):
        if kname(r["Kernel_Name"]) == "k_score_topk":
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    rows0 = bench.get("config", {}).get("units")  # round 0 scores every unit
    N = bench.get("config", {}).get("nodes")
    full = valu["kernels"]["k_score_topk"]["per_solve"]
    if rows0 and N and pairs and tot.get("SQ_INSTS_VALU"):
        p0 = float(rows0) * N
        split = {"source": "SQ pass of the no-select build (KP_FZ_EXP=1, round 0: units x nodes pairs) "
                           "vs the full kernel's SQ pass over the whole solve",
                 "pairs_no_select_run": p0, "pairs_full_solve": pairs,
                 "score_and_threshold": {"valu_lane_ops_per_pair": 64 * tot["SQ_INSTS_VALU"] / p0,
                                         "salu_per_pair_x64": 64 * tot.get("SQ_INSTS_SALU", 0) / p0,
                                         "lds_per_pair_x64": 64 * tot.get("SQ_INSTS_LDS", 0) / p0},
                 "whole_kernel": {"valu_lane_ops_per_pair": 64 * full["SQ_INSTS_VALU"] / pairs,
                                  "salu_per_pair_x64": 64 * full.get("SQ_INSTS_SALU", 0) / pairs,
                                  "lds_per_pair_x64": 64 * full.get("SQ_INSTS_LDS", 0) / pairs}}
        split["select"] = {k: split["whole_kernel"][k] - split["score_and_threshold"][k]
                           for k in split["whole_kernel"]}
        json.dump(split, open(os.path.join(prof, f"{rnd}_valu_split.json"), "w"), indent=1)
for name, obj in (("pmc", hbm), ("valu", valu), ("lds", lds)):
    if obj["kernels"]:
        json.dump(obj, open(os.path.join(prof, f"{rnd}_{name}.json"), "w"), indent=1)

# HIP runtime trace of kp_place: device allocations after the warm-up call
rt = os.path.join(src, "rt")
api = os.path.join(rt, "run_hip_api_trace.csv")
ktr = os.path.join(rt, "run_kernel_trace.csv")
if os.path.exists(api) and os.path.exists(ktr):
    kr = sorted(csv.DictReader(open(ktr)), key=lambda r: int(r["Start_Timestamp"]))
    fin = [int(r["End_Timestamp"]) for r in kr if "k_finalize" in r["Kernel_Name"]]
    ar = list(csv.DictReader(open(api)))
    names = ("hipMalloc", "hipFree", "hipMallocAsync", "hipFreeAsync", "hipHostMalloc", "hipHostFree")
    calls = [(r["Function"], int(r["Start_Timestamp"])) for r in ar if r.get("Function") in names]
    # between the end of the warm-up call and the end of the last timed call
    # (kp_destroy's frees come after it)
    after = [c for c in calls if len(fin) > 1 and fin[0] < c[1] <= fin[-1]]
    with open(os.path.join(prof, f"{rnd}_place_alloc_check.txt"), "w") as f:
        f.write("# HIP runtime trace of tools/place_steps.py: 1 warm-up kp_place + 3 timed kp_place\n")
        f.write(f"# kp_place calls seen (k_finalize launches): {len(fin)}\n")
        f.write(f"# device/host allocation API calls in the whole run: {len(calls)}\n")
        f.write(f"# ... inside the timed calls (after the warm-up's last kernel, up to the "
                f"last call's last kernel): {len(after)}\n")
        for fn, t in after:
            f.write(f"{fn} at {t}\n")
        log = os.path.join(rt, "place.log")
        if os.path.exists(log):
            f.write("".join(l for l in open(log) if l.startswith("place ")))
print("wrote profiles/%s_*" % rnd)
