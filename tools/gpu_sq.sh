# SQ counters of selected kernels (one --pmc pass, kernel trace only).
# usage: bash tools/gpu_sq.sh [kernel-regex] [out-suffix]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
RE=${1:-'k_accept|k_plan|k_score32|k_select_t'}
OUT=gpurun_out/sq${2:-}
rm -rf $OUT; mkdir -p $OUT
CTR=${SQ_CTR:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR}
timeout -s KILL 120 rocprofv3 --pmc $CTR \
  --kernel-include-regex "$RE" --output-format csv \
  -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 \
  > $OUT/p1.log 2>&1 || exit $?
echo sq ok
