# Same-box A/B of library builds (abl/<name>.so, built by
# ABOUT=$PWD/abl tools/build_variant.sh <rev> <name>; "cur" = the in-tree
# libkplace.so): config #3 solve (tools/cfg_time.py) alternated x3, then the
# config #4 solve (tools/c4_time.py) alternated x2. LIBS overrides the list.
set -o pipefail
OUT=${OUT:-gpurun_out/ab_libs}; mkdir -p $OUT
LIBS=${LIBS:-"base cur"}
lib_of() { [ "$1" = cur ] && echo "$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so" || echo "$PWD/abl/$1.so"; }
for i in 1 2 3; do for l in $LIBS; do
  KPLACE_LIB=$(lib_of $l) timeout -k 10 120 python3 tools/cfg_time.py >> $OUT/c3.txt 2>&1 || { tail -5 $OUT/c3.txt; exit 1; }
done; done
cat $OUT/c3.txt
if [ "$SKIP_C4" != 1 ]; then
for i in 1 2; do for l in $LIBS; do
  KPLACE_LIB=$(lib_of $l) timeout -k 10 180 python3 tools/c4_time.py >> $OUT/c4.txt 2>&1 || { tail -5 $OUT/c4.txt; exit 1; }
done; done
cat $OUT/c4.txt
fi
