# A/B of one library knob on the config #5 streaming loop (tools/stream_profile.py,
# 40 batches), alternating: bash tools/ab_stream_env.sh KP_ACC_WAVES "0 4096 2048"
set -o pipefail
export KP_DEBUG_KNOBS=1  # the library reads its A/B knobs only with this set
VAR=$1; VALS=$2
mkdir -p gpurun_out/abs
for i in 1 2; do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python -u tools/stream_profile.py 40 > gpurun_out/abs/${VAR}_$v.$i.log 2>&1 || exit $?
    echo "$VAR=$v $(grep solve gpurun_out/abs/${VAR}_$v.$i.log)"
  done
done
