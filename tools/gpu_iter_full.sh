# One development iteration: the whole -m gpu suite, a config #3 bench line
# (no kernel events) and the config #4 solve time.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/it_noev.json > gpurun_out/it_noev.log 2>&1 || { tail -20 gpurun_out/it_noev.log; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/it_noev.json'));print('config3 solve ms', round(b['ms_per_step'],2))"
timeout -k 10 300 python -u tools/c4_time.py 2>&1 | tail -1
