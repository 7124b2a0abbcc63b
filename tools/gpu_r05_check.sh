# r05: the whole -m gpu suite, score-matrix timings, the default bench line,
# and the score-matrix kernel's rocprofv3 stats + FETCH/WRITE PMC passes
set -o pipefail
OUT=gpurun_out/r05chk; rm -rf $OUT; mkdir -p $OUT/sm $OUT/pmc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for a in "" "--no-mask" "--no-score" ""; do timeout -k 10 120 python3 tools/score_dev_time.py $a >> $OUT/sd.txt 2>&1 || exit 1; done
cat $OUT/sd.txt
timeout -k 10 600 python -u bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print('bench', b['ms_per_step'], b['score_matrix']['frac'], b['score_matrix']['ms_per_call'], b['config4']['solve_ms'], b['config4']['preempt_ms'], b['phases'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sm -o run -- python3 tools/score_dev_time.py > $OUT/sm/score_dev.log 2>&1 || exit $?
echo sm ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'k_score32c' --output-format csv -d $OUT/pmc/$C -o run -- python3 tools/score_dev_time.py > $OUT/pmc/$C.log 2>&1 || exit $?
  echo "pmc $C ok"
done
rm -f $OUT/sm/run_kernel_trace.csv
