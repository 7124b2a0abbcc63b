# A/B of library builds / knobs on config #4 only (tools/c4_time.py), alternated
# N times: N=2 bash tools/ab_c4.sh lib_a lib_b@KNOB=v ...
set -o pipefail
export KP_DEBUG_KNOBS=1
AB=kubernetes-native-distributed-ai-job-scheduler_amd/build/ab
for i in $(seq 1 ${N:-2}); do
  for c in "$@"; do
    lib=${c%%@*}; envs=""
    [ "$c" != "$lib" ] && envs=$(echo "${c#*@}" | tr ',' ' ')
    echo -n "$c "
    env $envs KPLACE_LIB=$PWD/$AB/$lib.so timeout -k 10 200 python -u tools/c4_time.py 2>&1 | tail -1 || exit 1
  done
done
