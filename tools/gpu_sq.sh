# SQ counters of the pass kernels (one --pmc pass, kernel trace only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sq
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --kernel-include-regex 'k_accept|k_plan|k_score32|k_select_t' --output-format csv \
  -d gpurun_out/sq/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream \
  > gpurun_out/sq/p1.log 2>&1 || exit $?
echo sq ok
