# Kernel trace of the bench (no per-kernel events) for per-round analysis.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > gpurun_out/prof/bench.log 2>&1
echo "rocprof rc=$?"
