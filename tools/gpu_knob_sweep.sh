# Kernel-level sweep of one library knob (KP_DEBUG_KNOBS=1 $KNOB=v for v in
# VALS): rocprofv3 kernel stats of the config #3 solve (cfg_time.py) and, unless
# SKIP_C4=1, the config #4 solve (c4_time.py); per value the per-kernel totals
# (kstats_cmp.py). Output under $OUT.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/sweep}; rm -rf $OUT; mkdir -p $OUT
for v in $VALS; do
  for cfg in c3 c4; do
    [ "$cfg" = c4 ] && [ "$SKIP_C4" = 1 ] && continue
    script=tools/cfg_time.py; [ $cfg = c4 ] && script=tools/c4_time.py
    KP_DEBUG_KNOBS=1 env $KNOB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/$v.$cfg -o run -- python3 $script > $OUT/$v.$cfg.log 2>&1 || { tail -5 $OUT/$v.$cfg.log; exit 1; }
    tail -1 $OUT/$v.$cfg.log
    rm -f $OUT/$v.$cfg/run_kernel_trace.csv
  done
done
for cfg in c3 c4; do
  [ "$cfg" = c4 ] && [ "$SKIP_C4" = 1 ] && continue
  python3 tools/kstats_cmp.py $(for v in $VALS; do echo $OUT/$v.$cfg/run_kernel_stats.csv; done) 2>/dev/null | head -6 || true
done
