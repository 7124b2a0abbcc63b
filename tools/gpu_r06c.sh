# r06: the all-ties bisection test against the pre-fix library (expected to
# show the bug) and the fixed in-tree one, the whole GPU suite, then a same-box
# A/B of the pre-hygiene build (abl/r06_pre.so) vs the in-tree build
set -o pipefail
OUT=gpurun_out/r06c; rm -rf $OUT; mkdir -p $OUT
KPLACE_LIB=$PWD/abl/r06_pre.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "bisection_all_ties" > $OUT/pre_ties.log 2>&1
echo "pre-fix library, all-ties bisection: rc $?"; grep -E "passed|failed" $OUT/pre_ties.log | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pt_all.log 2>&1 || { tail -40 $OUT/pt_all.log; exit 1; }
tail -1 $OUT/pt_all.log
LIBS="r06_pre cur" OUT=$OUT bash tools/gpu_ab.sh
