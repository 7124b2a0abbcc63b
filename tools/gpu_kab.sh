# Kernel-level same-box A/B of library builds: rocprofv3 kernel stats of the
# config #3 solve (cfg_time.py, 6 solves) and the config #4 solve (c4_time.py)
# per build in LIBS (abl/<name>.so, "cur" = the in-tree library), summed per
# kernel by kstats_cmp.py. OUT names the output directory.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/kab}; mkdir -p $OUT
LIBS=${LIBS:-"base cur"}
lib_of() { [ "$1" = cur ] && echo "$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so" || echo "$PWD/abl/$1.so"; }
# REPS > 1: the config #3 runs repeated, alternating the builds (per-kernel
# totals then cover REPS x 6 solves of each build)
for rep in $(seq 1 ${REPS:-1}); do for l in $LIBS; do
  for cfg in c3 c4; do
    [ "$cfg" = c4 ] && [ "$rep" -gt 1 ] && continue
    [ "$cfg" = c4 ] && [ "$SKIP_C4" = 1 ] && continue
    script=tools/cfg_time.py; [ $cfg = c4 ] && script=tools/c4_time.py
    d=$OUT/$l.$cfg; [ "$rep" -gt 1 ] && d=$OUT/$l.$cfg.r$rep
    KPLACE_LIB=$(lib_of $l) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $d -o run -- python3 $script > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    tail -1 $d.log
  done
done; done
for l in $LIBS; do echo "== $l (config #3, second solve)"; python3 tools/ktrace_sum.py $OUT/$l.c3/run_kernel_trace.csv k_score_topk,k_merge_tour | tail -3; done
rm -f $OUT/*/run_kernel_trace.csv
for cfg in c3 c4; do
  [ "$cfg" = c4 ] && [ "$SKIP_C4" = 1 ] && continue
  python3 tools/kstats_cmp.py $(for l in $LIBS; do echo $OUT/$l.$cfg/run_kernel_stats.csv; done)
  [ "$cfg" = c3 ] && for rep in $(seq 2 ${REPS:-1}); do
    python3 tools/kstats_cmp.py $(for l in $LIBS; do echo $OUT/$l.$cfg.r$rep/run_kernel_stats.csv; done) 2>/dev/null | head -5 || true
  done
done
true  # the summaries above are informational: a failed run already exited
