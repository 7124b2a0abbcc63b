# r04: pass-kernel phase profile (KP_PASS_PROFILE builds, all rounds) of HEAD vs the working tree
set -o pipefail
mkdir -p gpurun_out/pp
for n in pp_head pp_wt pp_head pp_wt; do
  KPLACE_LIB=$PWD/ab/$n.so KP_DEBUG_KNOBS=1 KP_FZ_PROF=1 timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix > gpurun_out/pp/$n.log 2>&1 || exit $?
  echo "== $n"; grep "kp_pass_prof" gpurun_out/pp/$n.log
done
