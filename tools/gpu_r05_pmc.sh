# r05: the int32 VALU issue rate (tools/valu_peak), the LDS bank-conflict
# pass of the config #3 candidate phase, and SQ counters of the config #4
# pass kernels (one PMC group per rocprofv3 run).
set -o pipefail
OUT=gpurun_out/r05pmc; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 60 ./tools/valu_peak > $OUT/valu_peak.txt 2>&1 || exit 1
cat $OUT/valu_peak.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B1="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-score-matrix"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-include-regex 'k_score_topk|k_merge' --output-format csv -d $OUT/lds -o run -- python3 $B1 > $OUT/lds.log 2>&1 || exit $?
echo lds ok
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex 'k_plan|k_accept|k_score_topk' --output-format csv -d $OUT/sq4 -o run -- python3 tools/c4_time.py > $OUT/sq4.log 2>&1 || exit $?
echo sq4 ok
python3 - <<'PY'
import csv, collections, re
def agg(path):
    a = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = re.search(r"(k_\w+)", r["Kernel_Name"]).group(1)
        a[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return a
for name, p in (("lds", "gpurun_out/r05pmc/lds/run_counter_collection.csv"), ("sq4", "gpurun_out/r05pmc/sq4/run_counter_collection.csv")):
    for k, d in agg(p).items():
        print(name, k, {c: f"{v:.4g}" for c, v in d.items()})
PY
rm -f $OUT/*/run_kernel_trace.csv
