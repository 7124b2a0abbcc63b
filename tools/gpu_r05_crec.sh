# r05: the fused kernel's precomputed row records (KP_FZ_CREC) and the
# threshold merge (KP_MERGE_THR): parity, then same-box config #3 / #4
# timing of the knob settings and of the plan register-budget builds.
set -o pipefail
OUT=gpurun_out/r05crec; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or score_geometry or compaction or preempt or long_row or config or golden" -x -q --timeout 150 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -40 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > $OUT/ptl.log 2>&1 || { tail -40 $OUT/ptl.log; exit 1; }
tail -1 $OUT/ptl.log
export KP_DEBUG_KNOBS=1
for i in 1 2 3; do for kn in "KP_FZ_CREC=0 KP_MERGE_THR=0" "KP_FZ_CREC=1 KP_MERGE_THR=0" "KP_FZ_CREC=1 KP_MERGE_THR=1"; do env $kn timeout -k 10 120 python3 tools/cfg_time.py >> $OUT/c3.txt 2>&1 && echo "  ^ $kn" >> $OUT/c3.txt || exit 1; done; done
cat $OUT/c3.txt
for i in 1 2; do for kn in "KP_FZ_CREC=0 KP_MERGE_THR=0" "KP_FZ_CREC=1 KP_MERGE_THR=0" "KP_FZ_CREC=1 KP_MERGE_THR=1"; do env $kn timeout -k 10 180 python3 tools/c4_time.py >> $OUT/c4.txt 2>&1 && echo "  ^ $kn" >> $OUT/c4.txt || exit 1; done; done
cat $OUT/c4.txt
# plan register budget A/B (abl/base5 = this tree, plan7 / plan8 = KP_PLAN_WPE 7 / 8)
LIBS="base5 plan7 plan8" bash tools/gpu_r05_ab.sh > $OUT/plan_ab.txt 2>&1 || { tail -5 $OUT/plan_ab.txt; exit 1; }
cat $OUT/plan_ab.txt
