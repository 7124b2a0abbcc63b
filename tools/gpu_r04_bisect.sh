# r04: bisect the config #3 solve difference between the working tree and HEAD (ab/base.so)
set -o pipefail
mkdir -p gpurun_out/bis
B="--steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix"
for i in 1 2; do
  for v in default base_layout base; do
    case $v in
      default) L=; E= ;;
      nosum) L=; E="KP_DEBUG_KNOBS=1 KP_CSR_SUMMARY=0" ;;
      base_layout) L=$PWD/ab/base_layout.so; E= ;;
      base) L=$PWD/ab/base.so; E= ;;
    esac
    env $E KPLACE_LIB=$L timeout -k 10 120 python3 bench.py $B --out gpurun_out/bis/$v.$i.json > gpurun_out/bis/$v.$i.log 2>&1 || exit $?
    python3 -c "import json;b=json.load(open('gpurun_out/bis/$v.$i.json'));print('$v c3', round(b['ms_per_step'],3), b['config']['placed_jobs'])"
  done
done
