set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_accbig.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_accbig.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_accbig.log | head; exit $rc; }
bash tools/ab_c34.sh main big big@KP_ACC_BIG_RATIO=16 big@KP_ACC_BIG_RATIO=0
