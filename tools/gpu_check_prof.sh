set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1
  echo "bench rc=$?"
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof/bench.log 2>&1
  echo "rocprof rc=$?"
fi
