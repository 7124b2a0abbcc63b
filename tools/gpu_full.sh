# full -m gpu suite + the default bench line (the round-end driver's two steps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_full.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_full.log | head -20; exit $rc; }
timeout -k 10 900 python -u bench.py --out gpurun_out/bench_full.json > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/bench_full.json'));print('ms', b['ms_per_step'], 'c4', b['config4']['solve_ms'], b['config4']['preempt_ms'], 'stream p50', b['streaming']['p50_ms'])"
