# parity tests, then a bench line without CPU baseline / streaming, plus roofline microbench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --out gpurun_out/b_ev.json > gpurun_out/b_ev.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-kernel-events --out gpurun_out/b_noev.json > gpurun_out/b_noev.log 2>&1 || exit $?
python3 - <<'PY'
import json
for e in ("noev","ev"):
    b=json.load(open(f"gpurun_out/b_{e}.json"))
    t=b["roofline"]
    print(e, round(b["ms_per_step"],3), "ms", b["config"]["rounds"], b["config"]["passes"], b["config"]["placed_jobs"], "roof", round(t["frac"],3), "avg launch us", round(t["avg_launch_ms"]*1e3,1))
PY
true
