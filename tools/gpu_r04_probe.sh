# r04 probes: L2 persistence across kernel boundaries (tools/l2_persist.hip), and the
# pass-kernel phase profile of rounds >= 20 (KP_PASS_PROFILE build, one-wave accept).
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 60 ./tools/l2_persist > gpurun_out/r04/l2_persist.txt 2>&1; echo "l2 rc=$?"
cat gpurun_out/r04/l2_persist.txt
KPLACE_LIB=$PWD/ab/passprof20.so KP_DEBUG_KNOBS=1 KP_ACC_WG=0 KP_FZ_PROF=1 KP_PASS_SPANS=1 timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > gpurun_out/r04/spans20.log 2>&1
echo "spans rc=$?"
grep "kp_pass_prof" gpurun_out/r04/spans20.log
