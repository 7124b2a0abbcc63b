# Kernel traces of one bench solve under two env settings (A/B of a library
# knob): gpu_trace_ab.sh "VAR=a" "VAR=b" ; per-kernel totals via ktrace_sum.py
set -o pipefail
export KP_DEBUG_KNOBS=1  # the library reads its A/B knobs only with this set
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for setting in "$@"; do
  OUT=gpurun_out/trace_ab$i
  rm -rf $OUT; mkdir -p $OUT
  env $setting true || exit 2
  export $setting
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > $OUT/bench.log 2>&1 || exit $?
  echo "== $setting"
  python3 tools/ktrace_sum.py $OUT/run_kernel_trace.csv k_accept,k_plan || exit 1
  rm -f $OUT/run_kernel_trace.csv
  i=$((i+1))
done
