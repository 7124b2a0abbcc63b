# r06: config #4 plan cost of the long-row bid minima: the in-tree build vs
# timing-only variants (abl/bmin1: plain stores instead of atomics; bmin2: no
# minima at all) and the candidate fix (abl/bmin3: butterfly pre-reduction over
# the wave's slot groups, vector atomics), with bmin3's parity first
set -o pipefail
OUT=gpurun_out/r06e; rm -rf $OUT; mkdir -p $OUT
KPLACE_LIB=$PWD/abl/bmin3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread -k "long_row or config4 or bid_minima or fused_topk" > $OUT/pt_bmin3.log 2>&1 || { tail -30 $OUT/pt_bmin3.log; exit 1; }
tail -1 $OUT/pt_bmin3.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in cur bmin1 bmin2 bmin3; do
  if [ $v = cur ]; then L=; else L=$PWD/abl/$v.so; fi
  KPLACE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 tools/c4_time.py > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  grep "config4 solve" $OUT/$v.log
  python3 tools/kstat.py $OUT/$v/run_kernel_stats.csv 3 > $OUT/$v.kstat; head -5 $OUT/$v.kstat
  rm -f $OUT/$v/run_kernel_trace.csv
done
LIBS="cur bmin3" SKIP_C4=1 OUT=$OUT bash tools/gpu_ab.sh
