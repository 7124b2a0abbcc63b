# r06: k_score32c row body specialised (full tiles without store guards, rows
# without GPU request / affinity skip those compares, masks assembled in the
# variant's block): parity of both builds, then kp_score_dev timing alternated
# against the in-tree (pre-change) build
set -o pipefail
OUT=gpurun_out/r06g; rm -rf $OUT; mkdir -p $OUT
for v in sc6 sc0; do
  KPLACE_LIB=$PWD/abl/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread -k "score" > $OUT/pt_$v.log 2>&1 || { tail -30 $OUT/pt_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pt_$v.log)"
done
for i in 1 2 3; do for v in cur sc6 sc0; do
  if [ $v = cur ]; then L=; else L=$PWD/abl/$v.so; fi
  KPLACE_LIB=$L timeout -k 10 120 python3 tools/score_dev_time.py 2>&1 | sed "s/^/$v /" | tee -a $OUT/t.txt
done; done
