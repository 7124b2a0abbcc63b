# One iteration: parity tests, bench (no events), kernel-trace profile of the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/it_noev.json > gpurun_out/it_noev.log 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --out gpurun_out/it_ev.json > gpurun_out/it_ev.log 2>&1 || exit $?
python3 -c "import json;b=json.load(open('gpurun_out/it_noev.json'));e=json.load(open('gpurun_out/it_ev.json'));t=e['roofline'];print('solve', round(b['ms_per_step'],2),'ms (events', round(e['ms_per_step'],2),') frac',round(t['frac'],3),'avg us',round(t['avg_launch_ms']*1e3,1), b['config']['rounds'], b['config']['passes'], b['config']['placed_jobs'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof; mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > gpurun_out/prof/bench.log 2>&1
echo "rocprof rc=$?"
