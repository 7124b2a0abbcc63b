# Incremental candidate phase diagnostics: per-round changed / rescanned
# counts (KP_INCR_TRACE) for config #3 and #4, and kernel stats of both.
set -o pipefail
mkdir -p gpurun_out/incr
export KP_DEBUG_KNOBS=1
KP_INCR_TRACE=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/incr/b3.json > gpurun_out/incr/trace3.log 2>&1 || exit 1
KP_INCR_TRACE=1 timeout -k 10 200 python -u tools/c4_time.py > gpurun_out/incr/trace4.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/incr/p3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/incr/p3.json > gpurun_out/incr/p3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/incr/p4 -o run -- python3 tools/c4_time.py > gpurun_out/incr/p4.log 2>&1 || exit 1
rm -f gpurun_out/incr/p3/run_kernel_trace.csv gpurun_out/incr/p4/run_kernel_trace.csv
echo done
