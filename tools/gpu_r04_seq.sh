# r04: plan score-sequence member loop: pass parity tests, then A/B vs ab/base.so
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_seq.log 2>&1 || { tail -30 gpurun_out/r04/pytest_seq.log; exit 1; }
tail -1 gpurun_out/r04/pytest_seq.log
LIBS="lib ab/base.so" C4=1 bash tools/ab_libs.sh
# kernel-argument placement A/B (device-memory kernargs vs the runtime default)
for i in 1 2; do
  for kd in 0 1; do
    HIP_FORCE_DEV_KERNARG=$kd timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix --out gpurun_out/ab/kd$kd.$i.json > gpurun_out/ab/kd$kd.$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/ab/kd$kd.$i.json'));print('kernarg_dev=$kd', round(b['ms_per_step'],3))"
  done
done
