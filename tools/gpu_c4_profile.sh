# Config #4 per-kernel time and k_score_topk's VALU lane-ops per pair
# (tools/c4_time.py: 3 solves; summarised per solve into $OUT/summary.txt)
set -o pipefail
OUT=gpurun_out/c4_profile; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- python3 tools/c4_time.py > $OUT/ks.log 2>&1 || exit $?
rm -f $OUT/ks/run_kernel_trace.csv
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-include-regex k_score_topk --output-format csv -d $OUT/sq -o run -- python3 tools/c4_time.py > $OUT/sq.log 2>&1 || exit $?
python3 - > $OUT/summary.txt <<'PY'
import csv, re, collections
O = "gpurun_out/c4_profile"
log = open(f"{O}/ks.log").read()
m = re.search(r"pairs (\d+)", log)
pairs = int(m.group(1)) if m else None
print("# config #4 (tools/c4_time.py: 3 solves), rocprofv3 kernel stats per solve")
print("\n".join(l for l in log.splitlines() if "config4 solve ms" in l))
rows = sorted(csv.DictReader(open(f"{O}/ks/run_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    k = re.search(r"(k_\w+|__amd\w+)", r["Name"]); k = k.group(0) if k else r["Name"][:30]
    agg[k][0] += int(r["Calls"]); agg[k][1] += float(r["TotalDurationNs"])
tot = sum(v[1] for v in agg.values())
print(f"all kernels {tot / 3 / 1e6:.1f} ms per solve")
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{t / 3 / 1e6:9.2f} ms {c / 3:9.1f} launches  avg {t / max(c, 1) / 1e3:9.2f} us  {k}")
sq = collections.defaultdict(float)
for r in csv.DictReader(open(f"{O}/sq/run_counter_collection.csv")):
    sq[r["Counter_Name"]] += float(r["Counter_Value"])
print("# k_score_topk SQ counters (rocprofv3 --pmc, 3 solves)")
for k, v in sorted(sq.items()):
    print(f"{k} {v:.0f}")
if pairs:
    print(f"pairs per solve {pairs}")
    print(f"valu_lane_ops_per_pair {64 * sq['SQ_INSTS_VALU'] / 3 / pairs:.2f}")
    print(f"salu_per_pair_x64 {64 * sq['SQ_INSTS_SALU'] / 3 / pairs:.2f}")
    if sq.get("SQ_WAVE_CYCLES"):
        print(f"wait_any_frac {sq['SQ_WAIT_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}")
PY
rm -f $OUT/sq/run_counter_collection.csv $OUT/sq/run_kernel_trace.csv
cat $OUT/summary.txt
