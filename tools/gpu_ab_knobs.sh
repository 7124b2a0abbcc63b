# config #3 solve times (tools/cfg_time.py) of library builds x knob settings,
# alternated twice: CASES="lib@VAR=1,VAR2=2 lib2 ..." (lib = build/ab/<lib>.so or "main")
set -o pipefail
export KP_DEBUG_KNOBS=1
mkdir -p gpurun_out
AB=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/build/ab
for rep in 1 2; do
  for c in $CASES; do
    lib=${c%%@*}; kn=""; [ "$c" != "$lib" ] && kn=${c#*@}
    if [ "$lib" = main ]; then L=""; else L="KPLACE_LIB=$AB/$lib.so"; fi
    r=$(env $L ${kn//,/ } timeout -k 10 120 python tools/cfg_time.py 2>&1 | tail -1) || { echo "FAILED $c: $r"; exit 1; }
    echo "$c: $r"
  done
done
