# A/B of library builds on config #4's preemption (bench config4 leg, 2 steps), alternated 2x
set -o pipefail
export KP_DEBUG_KNOBS=1
mkdir -p gpurun_out/abp
AB=kubernetes-native-distributed-ai-job-scheduler_amd/build/ab
for i in 1 2; do
  for c in "$@"; do
    lib=${c%%@*}; envs=""
    [ "$c" != "$lib" ] && envs=$(echo "${c#*@}" | tr ',' ' ')
    n=$(echo "$c" | tr '@=,' '___')
    env $envs KPLACE_LIB=$PWD/$AB/$lib.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --place-steps 0 --no-kernel-events --c4-steps 2 --out gpurun_out/abp/$n.$i.json > gpurun_out/abp/$n.$i.log 2>&1 || { tail -5 gpurun_out/abp/$n.$i.log; exit 1; }
    python3 -c "import json;b=json.load(open('gpurun_out/abp/$n.$i.json'));c=b['config4'];print('$c', 'solve', round(c['solve_ms'],1), 'preempt', round(c['preempt_ms'],2))"
  done
done
