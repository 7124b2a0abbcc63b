# r04: score matrix A/B on one box: rows per kp_score_dev launch (all vs cap_U-sized chunks), vs HEAD
set -o pipefail
export KP_DEBUG_KNOBS=1
for i in 1 2; do
  for ch in 0 26525 50000; do
    echo "chunk $ch"
    KP_SCORE_DEV_CHUNK=$ch timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
  done
  KPLACE_LIB=$PWD/ab/sm_head.so timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
done
