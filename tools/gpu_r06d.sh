# r06: where config #4's k_plan time goes: kernel stats with the long-row bid
# minima on (default) and off (KP_BMIN_WIN=1e6: no plan atomics), and the
# SQ counters of k_plan / k_accept
set -o pipefail
OUT=gpurun_out/r06d; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export KP_DEBUG_KNOBS=1
for v in def nobmin; do
  if [ $v = nobmin ]; then export KP_BMIN_WIN=1000000; else unset KP_BMIN_WIN; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 tools/c4_time.py > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  grep "config4 solve" $OUT/$v.log
  python3 tools/kstat.py $OUT/$v/run_kernel_stats.csv 4 | head -8
  rm -f $OUT/$v/run_kernel_trace.csv
done
unset KP_BMIN_WIN
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_plan|k_accept" --output-format csv -d $OUT/sq -o run -- python3 tools/c4_time.py > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
python3 - <<'PY'
import csv, collections, re
sq = collections.defaultdict(float)
for r in csv.DictReader(open("gpurun_out/r06d/sq/run_counter_collection.csv")):
    k = "k_plan" if "k_plan" in r["Kernel_Name"] else "k_accept"
    sq[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for k in ("k_plan", "k_accept"):
    d = {c: v for (kk, c), v in sq.items() if kk == k}
    print(k, {c: f"{v:.3g}" for c, v in sorted(d.items())})
    if d.get("SQ_WAVE_CYCLES"):
        print(k, "wait_any", round(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 3), "wait_inst", round(d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"], 3),
              "active_inst", round(d["SQ_ACTIVE_INST_ANY"] / d["SQ_WAVE_CYCLES"], 3), "valu/wave", round(d["SQ_INSTS_VALU"] / d["SQ_WAVES"], 1),
              "salu/wave", round(d["SQ_INSTS_SALU"] / d["SQ_WAVES"], 1), "cycles/wave", round(d["SQ_WAVE_CYCLES"] / d["SQ_WAVES"], 0))
PY
rm -f $OUT/sq/run_counter_collection.csv $OUT/sq/run_kernel_trace.csv
