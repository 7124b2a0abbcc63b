# Per-kernel time of the config #3 bench steps (rocprofv3 --kernel-trace
# --stats) for each library build in LIBS ("lib" = in-tree), summarised by
# tools/kstats_cmp.py: which kernel a change made faster or slower.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ks
LIBS=${LIBS:-"lib ab/base.so"}
for lib in $LIBS; do
  if [ "$lib" = lib ]; then n=lib; L=; else n=$(basename $lib .so); L=$PWD/$lib; fi
  KPLACE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks/$n -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix --out gpurun_out/ks/$n.json > gpurun_out/ks/$n.log 2>&1 || exit $?
  rm -f gpurun_out/ks/$n/run_kernel_trace.csv
done
python3 tools/kstats_cmp.py $(for lib in $LIBS; do if [ "$lib" = lib ]; then echo gpurun_out/ks/lib/run_kernel_stats.csv; else echo gpurun_out/ks/$(basename $lib .so)/run_kernel_stats.csv; fi; done)
