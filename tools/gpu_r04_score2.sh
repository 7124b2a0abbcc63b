# r04: k_score32c variants (knobs) on kp_score_dev, config #3 full queue
set -o pipefail
export KP_DEBUG_KNOBS=1
for i in 1 2; do
  timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
  timeout -k 10 120 python3 tools/score_dev_time.py --no-mask || exit $?
  timeout -k 10 120 python3 tools/score_dev_time.py --no-score || exit $?
  KP_SCORE_NPL=4 timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
  KP_SCORE_WG_TARGET=16384 timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
  KP_SCORE_MIN_RPB=16 KP_SCORE_WG_TARGET=100000 timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
  KP_SCORE_CLASSES=0 timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
done
