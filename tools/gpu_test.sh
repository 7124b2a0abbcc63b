# GPU parity suite (+ a short bench line): one development iteration.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 180 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/it_noev.json > gpurun_out/it_noev.log 2>&1 || { tail -20 gpurun_out/it_noev.log; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/it_noev.json'));print('solve ms', round(b['ms_per_step'],2), b['config'])"
