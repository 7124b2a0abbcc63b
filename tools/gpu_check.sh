set -o pipefail
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m1 gfx950 > gpurun_out/arch.txt || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1
  echo "bench rc=$?"
fi
