# One GPU call: parity tests, bench line, rocprofv3 kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out/prof
rocminfo 2>/dev/null | grep -m1 gfx950 > gpurun_out/arch.txt || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --out gpurun_out/bench1.json > gpurun_out/bench1.log 2>&1 || exit $?
echo "bench ok"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream --out gpurun_out/prof/bench_prof.json > gpurun_out/prof/bench.log 2>&1
echo "rocprof rc=$?"
