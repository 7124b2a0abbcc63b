# A/B timing of one library-tuning environment knob in ONE GPU call:
#   bash tools/ab_env.sh KP_ACC_WAVES "0 1024 4096"
# every value is run alternately, 3 times each, bench without events; with
# EVENTS=1 also a run with per-launch HIP events (filter+score roofline fraction).
set -o pipefail
export KP_DEBUG_KNOBS=1  # the library reads its A/B knobs only with this set
VAR=$1; VALS=$2
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for v in $VALS; do
    n=${VAR}_$v
    env $VAR=$v timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/ab/$n.$i.json > gpurun_out/ab/$n.$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/ab/$n.$i.json'));print('$n', round(b['ms_per_step'],3), b['config']['rounds'], b['config']['passes'], b['config']['placed_jobs'])"
    if [ "$EVENTS" = 1 ]; then
      env $VAR=$v timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --out gpurun_out/ab/$n.ev$i.json > gpurun_out/ab/$n.ev$i.log 2>&1 || exit $?
      python3 -c "import json;t=json.load(open('gpurun_out/ab/$n.ev$i.json'))['roofline'];print('$n', 'frac', round(t['frac'],3), 'avg us', round(t['avg_launch_ms']*1e3,1))"
    fi
  done
done
