# A/B timing of alternative library builds in ONE GPU call (same box): every
# ab/*.so (LIBS overrides: space-separated paths; "lib" = the in-tree build) is
# run alternately, 3 times each: config #3 bench solve without events, and with
# C4=1 also the config #4 solve (tools/c4_time.py).
set -o pipefail
mkdir -p gpurun_out/ab
LIBS=${LIBS:-"lib $(ls ab/*.so 2>/dev/null | grep -v passprof)"}
for i in $(seq 1 ${ITER:-3}); do
  for lib in $LIBS; do
    if [ "$lib" = lib ]; then n=lib; L=; else n=$(basename $lib .so); L=$PWD/$lib; fi
    KPLACE_LIB=$L timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix --out gpurun_out/ab/$n.$i.json > gpurun_out/ab/$n.$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/ab/$n.$i.json'));print('$n', round(b['ms_per_step'],3), b['config']['rounds'], b['config']['passes'], b['config']['placed_jobs'])"
    if [ "$C4" = 1 ]; then KPLACE_LIB=$L timeout -k 10 300 python3 tools/c4_time.py || exit $?; fi
  done
done
