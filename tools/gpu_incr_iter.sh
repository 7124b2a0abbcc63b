set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_incr.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_incr.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_incr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/it_noev.json > gpurun_out/it_noev.log 2>&1 || { tail -20 gpurun_out/it_noev.log; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/it_noev.json'));print('solve ms', round(b['ms_per_step'],2), b['config'])"
timeout -k 10 300 python -u tools/c4_time.py > gpurun_out/c4_time.txt 2>&1; cat gpurun_out/c4_time.txt
