# r04: class-form score matrix after the row specialisation: its parity tests, then timing
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "score" --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_sm.log 2>&1 || { tail -30 gpurun_out/r04/pytest_sm.log; exit 1; }
tail -1 gpurun_out/r04/pytest_sm.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
  timeout -k 10 120 python3 tools/score_dev_time.py --no-mask || exit $?
  timeout -k 10 120 python3 tools/score_dev_time.py --no-score || exit $?
done
