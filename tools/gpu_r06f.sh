# r06: k_plan with the long-row bid minima combined per workgroup (large
# rounds): parity (forced into every round too), then config #4 kernel stats
# and a same-box A/B against the r06 base build (abl/base.so)
set -o pipefail
OUT=gpurun_out/r06f; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 300 --timeout-method thread -k "long_row or config4 or bid_minima or fused_topk" > $OUT/pt.log 2>&1 || { tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o run -- python3 tools/c4_time.py > $OUT/ks.log 2>&1 || { tail -5 $OUT/ks.log; exit 1; }
grep "config4 solve" $OUT/ks.log
python3 tools/kstat.py $OUT/ks/run_kernel_stats.csv 3 > $OUT/ks.kstat; head -6 $OUT/ks.kstat
rm -f $OUT/ks/run_kernel_trace.csv
LIBS="base cur" OUT=$OUT bash tools/gpu_ab.sh
