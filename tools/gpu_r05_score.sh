set -o pipefail
OUT=gpurun_out/r05b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "score" -x -q --timeout 120 --timeout-method thread > $OUT/pt_score.log 2>&1 || { tail -30 $OUT/pt_score.log; exit 1; }
tail -2 $OUT/pt_score.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "score_dev" -x -q -s --timeout 200 --timeout-method thread > $OUT/pt_large.log 2>&1 || { tail -30 $OUT/pt_large.log; exit 1; }
grep -E "kp_score_dev|passed|failed" $OUT/pt_large.log
for a in "" "--no-mask" "--no-score" "" ; do timeout -k 10 120 python3 tools/score_dev_time.py $a >> $OUT/sd.txt 2>&1 || exit 1; done
cat $OUT/sd.txt
