# r05 development iteration (one GPU call): the score-matrix parity tests, the
# compaction / preemption paths, the full-size kp_score_dev digest test, the
# bench multi-rank rehearsal (config #4 + phase split), score-matrix timings.
# PYTEST_K narrows the parity step; SKIP_REHEARSAL=1 skips step 4.
set -o pipefail
OUT=gpurun_out/r05it; rm -rf $OUT; mkdir -p $OUT
K=${PYTEST_K:-"score or compaction or preempt or abi"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -k "$K" -x -v --timeout 150 --timeout-method thread > $OUT/pt_parity.log 2>&1 || { tail -40 $OUT/pt_parity.log; exit 1; }
tail -1 $OUT/pt_parity.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "score_dev" -x -v -s --timeout 250 --timeout-method thread > $OUT/pt_large.log 2>&1 || { tail -30 $OUT/pt_large.log; exit 1; }
grep -E "kp_score_dev|passed|failed" $OUT/pt_large.log
if [ "$SKIP_REHEARSAL" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_multi.py -x -v -s --timeout 550 --timeout-method thread > $OUT/pt_multi.log 2>&1 || { tail -40 $OUT/pt_multi.log; exit 1; }
  tail -1 $OUT/pt_multi.log
fi
for a in "" "--no-mask" "--no-score" ""; do timeout -k 10 120 python3 tools/score_dev_time.py $a >> $OUT/sd.txt 2>&1 || exit 1; done
cat $OUT/sd.txt
