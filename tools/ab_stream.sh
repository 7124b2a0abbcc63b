# A/B of build/ab/*.so on the streaming loop (tools/stream_profile.py), alternating.
set -o pipefail
for i in 1 2; do
  for lib in kubernetes-native-distributed-ai-job-scheduler_amd/build/ab/*.so; do
    n=$(basename $lib .so)
    KPLACE_LIB=$PWD/$lib timeout -k 10 200 python -u tools/stream_profile.py 30 > gpurun_out/abs_$n.$i.log 2>&1 || exit $?
    echo "$n $(grep solve gpurun_out/abs_$n.$i.log)"
  done
done
