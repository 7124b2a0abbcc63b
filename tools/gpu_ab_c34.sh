# config #3 and #4 solve times of library builds, alternated: LIBS="main base"
set -o pipefail
AB=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/build/ab
for rep in 1 2; do
  for lib in $LIBS; do
    if [ "$lib" = main ]; then L=""; else L="KPLACE_LIB=$AB/$lib.so"; fi
    r3=$(env $L timeout -k 10 120 python tools/cfg_time.py 2>&1 | tail -1) || { echo "FAILED $lib: $r3"; exit 1; }
    r4=$(env $L timeout -k 10 300 python tools/c4_time.py 2>&1 | tail -1) || { echo "FAILED c4 $lib: $r4"; exit 1; }
    echo "$lib | $r3 | $r4"
  done
done
