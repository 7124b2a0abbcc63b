# A/B of library builds / knobs on config #3 only (bench solve, no events),
# alternated N times: N=4 bash tools/ab_c3.sh lib_a lib_b@KNOB=v ...
set -o pipefail
export KP_DEBUG_KNOBS=1
mkdir -p gpurun_out/ab
AB=kubernetes-native-distributed-ai-job-scheduler_amd/build/ab
for i in $(seq 1 ${N:-4}); do
  for c in "$@"; do
    lib=${c%%@*}; envs=""
    [ "$c" != "$lib" ] && envs=$(echo "${c#*@}" | tr ',' ' ')
    n=$(echo "$c" | tr '@=,' '___')
    env $envs KPLACE_LIB=$PWD/$AB/$lib.so timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --out gpurun_out/ab/$n.$i.json > gpurun_out/ab/$n.$i.log 2>&1 || { tail -5 gpurun_out/ab/$n.$i.log; exit 1; }
    python3 -c "import json;b=json.load(open('gpurun_out/ab/$n.$i.json'));print('$c c3', round(b['ms_per_step'],3), b['config']['rounds'], b['config']['passes'])"
  done
done
