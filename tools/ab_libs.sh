# A/B timing of alternative library builds in ONE GPU call (same box):
# every build/ab/*.so is run alternately, 3 times each, bench without events.
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for lib in kubernetes-native-distributed-ai-job-scheduler_amd/build/ab/*.so; do
    n=$(basename $lib .so)
    KPLACE_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/ab/$n.$i.json > gpurun_out/ab/$n.$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/ab/$n.$i.json'));print('$n', round(b['ms_per_step'],3), b['config']['rounds'], b['config']['passes'], b['config']['placed_jobs'])"
  done
done
