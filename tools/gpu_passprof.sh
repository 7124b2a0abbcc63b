set -o pipefail
mkdir -p gpurun_out/pp
KP_DEBUG_KNOBS=1 KP_FZ_PROF=1 KPLACE_LIB=$PWD/abl/passprof.so SOLVES=2 timeout -k 10 300 python3 tools/cfg_time.py > gpurun_out/pp/c3.log 2>&1 || { tail -5 gpurun_out/pp/c3.log; exit 1; }
grep "kp_pass_prof\|solve ms" gpurun_out/pp/c3.log
