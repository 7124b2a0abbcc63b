# r05: the fused candidate phase's tile forms — parity (every fused test at
# both tile widths), then same-box timing of config #3 / #4 with
# KP_FZ_WAVES=8 and 16 and the library builds in abl/ (LIBS).
set -o pipefail
OUT=gpurun_out/r05fz; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or score_geometry or compaction" -x -q --timeout 150 --timeout-method thread > $OUT/pt.log 2>&1 || { tail -40 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
export KP_DEBUG_KNOBS=1
cur=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so
for i in 1 2 3; do
  for l in ${LIBS:-r04}; do KPLACE_LIB=$PWD/abl/$l.so timeout -k 10 120 python3 tools/cfg_time.py >> $OUT/c3.txt 2>&1 || exit 1; done
  for wv in 8 16; do KP_FZ_WAVES=$wv KPLACE_LIB=$cur timeout -k 10 120 python3 tools/cfg_time.py >> $OUT/c3.txt 2>&1 && echo "  ^ waves $wv" >> $OUT/c3.txt || exit 1; done
done
cat $OUT/c3.txt
for i in 1 2; do
  for l in ${LIBS:-r04}; do KPLACE_LIB=$PWD/abl/$l.so timeout -k 10 180 python3 tools/c4_time.py >> $OUT/c4.txt 2>&1 || exit 1; done
  for wv in 8 16; do KP_FZ_WAVES=$wv KPLACE_LIB=$cur timeout -k 10 180 python3 tools/c4_time.py >> $OUT/c4.txt 2>&1 && echo "  ^ waves $wv" >> $OUT/c4.txt || exit 1; done
done
cat $OUT/c4.txt
