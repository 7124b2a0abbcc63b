# r05: rocprofv3 kernel stats of the config #3 solves (tools/cfg_time.py, 6
# solves) and the config #4 solves (tools/c4_time.py, 3) for each library in
# LIBS (abl/<name>.so; "cur" = the in-tree build), summarised per solve by
# tools/kstats_cmp.py.
set -o pipefail
OUT=gpurun_out/r05ks; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in ${LIBS:-r04 cur}; do
  lib=$PWD/abl/$l.so; [ "$l" = cur ] && lib=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so
  KPLACE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_$l -o run -- python3 tools/cfg_time.py > $OUT/c3_$l.log 2>&1 || exit $?
  [ "$SKIP_C4" = 1 ] || KPLACE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_$l -o run -- python3 tools/c4_time.py > $OUT/c4_$l.log 2>&1 || exit $?
  rm -f $OUT/*_$l/run_kernel_trace.csv
  echo "$l ok"
done
for c in c3 c4; do
  for l in ${LIBS:-r04 cur}; do
    [ -f $OUT/${c}_$l/run_kernel_stats.csv ] || continue
    echo "== $c $l: $(tail -1 $OUT/${c}_$l.log)"
    python3 -c "
import csv,re,sys
n=6 if '$c'=='c3' else 3
rows=sorted(csv.DictReader(open('$OUT/${c}_$l/run_kernel_stats.csv')),key=lambda r:-float(r['TotalDurationNs']))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print(f'  all kernels {tot/n/1e3:9.1f} us per solve')
for r in rows[:9]:
    m=re.search(r'(k_\w+|rocprim\w*|__amd\w+)',r['Name']); k=m.group(0) if m else r['Name'][:30]
    print(f'  {float(r[\"TotalDurationNs\"])/n/1e3:9.1f} us {int(r[\"Calls\"])/n:7.1f} calls  avg {float(r[\"AverageNs\"])/1e3:7.2f} us  {k}')
"
  done
done
