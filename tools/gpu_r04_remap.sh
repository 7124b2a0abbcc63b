# r04: XCD-aware k_score_topk mapping (in-tree build) vs ab/base.so: config #3/#4
# timing alternated, and FETCH_SIZE of k_score_topk for both.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused or config3 or random" --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_remap.log 2>&1 || { tail -20 gpurun_out/r04/pytest_remap.log; exit 1; }
tail -1 gpurun_out/r04/pytest_remap.log
LIBS="lib ab/base.so" C4=1 bash tools/ab_libs.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B1="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events"
for v in lib base; do
  L=; [ $v = base ] && L=$PWD/ab/base.so
  for c in FETCH_SIZE WRITE_SIZE; do
    KPLACE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex k_score_topk --output-format csv -d gpurun_out/r04/pmc_$v$c -o run -- python3 $B1 > gpurun_out/r04/pmc_$v$c.log 2>&1 || exit $?
    python3 tools/pmc_fetch.py gpurun_out/r04/pmc_$v$c/run_counter_collection.csv | sed "s/^/$v /"
  done
done
