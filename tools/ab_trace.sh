# Kernel traces of alternative library builds (build/ab/*.so) in ONE GPU call:
# per build, the first launches of the named kernels (tools/ktrace_sum.py).
# usage: bash tools/ab_trace.sh [kernel,kernel,...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in kubernetes-native-distributed-ai-job-scheduler_amd/build/ab/*.so; do
  n=$(basename $lib .so)
  OUT=gpurun_out/abtr/$n
  rm -rf $OUT; mkdir -p $OUT
  KPLACE_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > $OUT/bench.log 2>&1 || exit $?
  echo "== $n"; python3 tools/ktrace_sum.py $OUT/run_kernel_trace.csv ${1:-k_score_topk,k_merge_topk} | tail -2
done
