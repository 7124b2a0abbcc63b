# r04: window bid minima only for long bidder rows (KP_BMIN_WIN windows) — A/B
# of the threshold (config #3 bench solve, config #4 solve) against HEAD's build
set -o pipefail
mkdir -p gpurun_out/bmin
B="--steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix"
for i in 1 2; do
  for v in 64 128 256 512; do
    if [ $v = base ]; then L=$PWD/ab/base.so; E=; else L=; E="KP_DEBUG_KNOBS=1 KP_BMIN_WIN=$v"; fi
    env $E KPLACE_LIB=$L timeout -k 10 120 python3 bench.py $B --out gpurun_out/bmin/$v.$i.json > gpurun_out/bmin/$v.$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/bmin/$v.$i.json'));print('win $v c3', round(b['ms_per_step'],3), b['config']['placed_jobs'])"
    env $E KPLACE_LIB=$L timeout -k 10 300 python3 tools/c4_time.py || exit $?
  done
done
