# Round evidence in one GPU call: full GPU test suite, the default bench line,
# a rocprofv3 kernel-trace/stats profile of the bench command, and the
# FETCH_SIZE / WRITE_SIZE PMC passes of the filter+score / select kernels.
set -o pipefail
OUT=gpurun_out/evidence
rm -rf $OUT; mkdir -p $OUT/prof $OUT/pmc
rocminfo 2>/dev/null | grep -m1 gfx950 > $OUT/arch.txt || true
[ "$SKIP_TESTS" = 1 ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
[ "$SKIP_TESTS" = 1 ] || tail -1 $OUT/pytest_gpu.log
[ "$SKIP_BENCH" = 1 ] || timeout -k 10 400 python -u bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1 || exit $?
echo bench ok
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream --out $OUT/prof/bench_prof.json > $OUT/prof/bench.log 2>&1 || exit $?
echo prof ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'k_score|k_select' --output-format csv \
    -d $OUT/pmc/$C -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream \
    > $OUT/pmc/$C.log 2>&1 || exit $?
  echo "$C ok"
done
