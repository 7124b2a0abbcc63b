# A/B of alternative library builds in ONE GPU call: per build/ab/*.so, the
# solve time without events and the filter+score roofline fraction with
# per-launch HIP events (bench.py), alternated 2 times.
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
  for lib in kubernetes-native-distributed-ai-job-scheduler_amd/build/ab/*.so; do
    n=$(basename $lib .so)
    KPLACE_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/ab/$n.$i.json > gpurun_out/ab/$n.$i.log 2>&1 || exit $?
    KPLACE_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --out gpurun_out/ab/$n.ev$i.json > gpurun_out/ab/$n.ev$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/ab/$n.$i.json'));e=json.load(open('gpurun_out/ab/$n.ev$i.json'));t=e['roofline'];print('$n', round(b['ms_per_step'],3), 'frac', round(t['frac'],3), 'avg us', round(t['avg_launch_ms']*1e3,1), b['config']['rounds'], b['config']['passes'], b['config']['placed_jobs'])"
  done
done
