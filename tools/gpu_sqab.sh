# SQ counter passes of k_score_topk for library builds (LIBS, abl/<name>.so or
# "cur"), config #3 (tools/cfg_time.py: 6 solves); two passes of 8 counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/sqab}; rm -rf $OUT; mkdir -p $OUT
LIBS=${LIBS:-"cur"}
RE=${RE:-k_score_topk}
lib_of() { [ "$1" = cur ] && echo "$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so" || echo "$PWD/abl/$1.so"; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LEVEL_WAVES SQ_INSTS_VALU"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_INSTS_SALU"
for l in $LIBS; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    KPLACE_LIB=$(lib_of $l) timeout -s KILL 180 rocprofv3 --pmc $P --kernel-include-regex "$RE" --output-format csv \
      -d $OUT/$l.p$i -o run -- python3 tools/cfg_time.py > $OUT/$l.p$i.log 2>&1 || { tail -5 $OUT/$l.p$i.log; exit 1; }
  done
done
python3 - $OUT $LIBS <<'PY'
import csv, collections, sys, glob
out, libs = sys.argv[1], sys.argv[2:]
for l in libs:
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{out}/{l}.p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(l, " ".join(f"{k}={v:.4g}" for k, v in sorted(agg.items())))
PY
