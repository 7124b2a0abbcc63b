set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -v -k "preempt or config4" --timeout 300 --timeout-method thread > gpurun_out/pytest_pre.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_pre.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --place-steps 0 --no-kernel-events --c4-steps 2 --out gpurun_out/b_pre.json > gpurun_out/b_pre.log 2>&1 || { tail -5 gpurun_out/b_pre.log; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/b_pre.json'));c=b['config4'];print('c4 solve',c['solve_ms'],'preempt',c['preempt_ms'])"
