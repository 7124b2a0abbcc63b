set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "pass_wg" --timeout 300 --timeout-method thread > gpurun_out/pytest_wg.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_wg.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_wg.log | head; exit $rc; }
bash tools/ab_c34.sh main main@KP_PASS_WG_T=128 main@KP_PASS_WG_T=256 main@KP_PASS_WG_T=512
