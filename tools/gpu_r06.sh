# r06 investigations, one mode per GPU call (tools/README.md):
#   rccl      the one-rank RCCL tests under rocprofv3 --rccl-trace
#             (profiles/r06_rccl_trace.txt) + the config #3 per-round pass table
#             (profiles/r06_c3_round_passes.txt)
#   bmin      config #4 kernel stats with the long-row bid minima on / off and
#             the SQ counters of k_plan / k_accept
#   score32c  kp_score_dev of abl/*.so builds (LIBS) against the in-tree
#             library, alternated x3, their parity first
set -o pipefail
MODE=${1:?mode}
OUT=gpurun_out/r06_$MODE; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case $MODE in
rccl)
  mkdir -p $OUT/rccl $OUT/c3
  timeout -k 10 170 rocprofv3 --rccl-trace --kernel-trace --stats --output-format csv -d $OUT/rccl -o run -- python3 -m pytest tests/test_gpu_rccl.py -m gpu -x -q -k "rank_config3_full or rank_config4" > $OUT/rccl/pytest.log 2>&1 || { tail -30 $OUT/rccl/pytest.log; exit 1; }
  python3 tools/rccl_summary.py $OUT/rccl | tee $OUT/rccl_summary.txt
  rm -f $OUT/rccl/run_kernel_trace.csv
  timeout -k 10 170 rocprofv3 --kernel-trace --output-format csv -d $OUT/c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --no-config2 --place-steps 0 --no-score-matrix --no-phases > $OUT/c3/bench.log 2>&1 || { tail -20 $OUT/c3/bench.log; exit 1; }
  python3 tools/c3_round_passes.py $OUT/c3/run_kernel_trace.csv > $OUT/round_passes.txt && tail -7 $OUT/round_passes.txt
  rm -f $OUT/c3/run_kernel_trace.csv ;;
bmin)
  export KP_DEBUG_KNOBS=1
  for v in def nobmin; do
    if [ $v = nobmin ]; then export KP_BMIN_WIN=1000000; else unset KP_BMIN_WIN; fi
    timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 tools/c4_time.py > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
    grep "config4 solve" $OUT/$v.log
    python3 tools/kstat.py $OUT/$v/run_kernel_stats.csv 3 > $OUT/$v.kstat; head -6 $OUT/$v.kstat
    rm -f $OUT/$v/run_kernel_trace.csv
  done
  unset KP_BMIN_WIN
  timeout -s KILL 170 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_plan|k_accept" --output-format csv -d $OUT/sq -o run -- python3 tools/c4_time.py > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
  rm -f $OUT/sq/run_kernel_trace.csv ;;
score32c)
  LIBS=${LIBS:-$(cd abl && ls *.so | sed 's/\.so$//')}
  for v in $LIBS; do
    KPLACE_LIB=$PWD/abl/$v.so timeout -k 10 170 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 150 --timeout-method thread -k "score" > $OUT/pt_$v.log 2>&1 || { tail -30 $OUT/pt_$v.log; exit 1; }
    echo "$v: $(tail -1 $OUT/pt_$v.log)"
  done
  for i in 1 2 3; do for v in cur $LIBS; do
    if [ $v = cur ]; then L=; else L=$PWD/abl/$v.so; fi
    KPLACE_LIB=$L timeout -k 10 120 python3 tools/score_dev_time.py 2>&1 | sed "s/^/$v /" | tee -a $OUT/t.txt
  done; done ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
