# r04: class-form score matrix, rows per workgroup via KP_SCORE_WG_TARGET (dynamic LDS records)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "score" --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_sm.log 2>&1 || { tail -30 gpurun_out/r04/pytest_sm.log; exit 1; }
tail -1 gpurun_out/r04/pytest_sm.log
export KP_DEBUG_KNOBS=1
for i in 1 2; do
  for t in 4096 2048 1024; do
    echo "wg_target $t"
    KP_SCORE_WG_TARGET=$t timeout -k 10 120 python3 tools/score_dev_time.py || exit $?
    KP_SCORE_WG_TARGET=$t timeout -k 10 120 python3 tools/score_dev_time.py --no-mask || exit $?
  done
done
