# config #5 streaming p50/p99 per knob setting, alternated N times:
# N=2 bash tools/ab_stream.sh KP_INCR=0 KP_INCR=1 ...
set -o pipefail
export KP_DEBUG_KNOBS=1
mkdir -p gpurun_out/ab
for i in $(seq 1 ${N:-2}); do
  for c in "$@"; do
    n=$(echo "$c" | tr '=,' '__')
    env $(echo "$c" | tr ',' ' ') timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/ab/stream_$n.$i.json > gpurun_out/ab/stream_$n.$i.log 2>&1 || { tail -5 gpurun_out/ab/stream_$n.$i.log; exit 1; }
    python3 -c "import json;b=json.load(open('gpurun_out/ab/stream_$n.$i.json'));s=b['streaming'];print('$c streaming p50', round(s['p50_ms'],3), 'p99', round(s['p99_ms'],3), {k:round(v,3) for k,v in s.items() if 'solve' in k and isinstance(v,float)})"
  done
done
