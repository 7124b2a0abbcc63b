set -o pipefail
mkdir -p gpurun_out/r06a
export KP_TIMEOUT=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a/pt_rccl.log 2>&1 || { tail -40 gpurun_out/r06a/pt_rccl.log; exit 1; }
tail -3 gpurun_out/r06a/pt_rccl.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a/pt_all.log 2>&1 || { tail -40 gpurun_out/r06a/pt_all.log; exit 1; }
tail -3 gpurun_out/r06a/pt_all.log
