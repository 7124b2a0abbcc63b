# Host-followed passes (KP_PASS_FOLLOW = M, default 2): full GPU suite with the
# default, then config #3 / #4 A/B against M = 0 (every round enqueues
# max_passes) and M = 3, and config #5 streaming p50/p99 for M = 0 and 2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_follow.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_follow.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_follow.log | head; exit $rc; }
bash tools/ab_c34.sh main@KP_PASS_FOLLOW=0 main main@KP_PASS_FOLLOW=3 || exit 1
export KP_DEBUG_KNOBS=1
for m in 0 2; do
  KP_PASS_FOLLOW=$m timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/ab/stream_$m.json > gpurun_out/ab/stream_$m.log 2>&1 || { tail -5 gpurun_out/ab/stream_$m.log; exit 1; }
  python3 -c "import json;b=json.load(open('gpurun_out/ab/stream_$m.json'));s=b['streaming'];print('follow $m streaming p50', round(s['p50_ms'],3), 'p99', round(s['p99_ms'],3))"
done
