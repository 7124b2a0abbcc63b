# Config #5 streaming A/B of library builds (abl/<name>.so, "cur" = in
# tree) alternated x2, then rocprofv3 kernel stats of the current build.
set -o pipefail
OUT=gpurun_out/stream_ab; rm -rf $OUT; mkdir -p $OUT
for i in 1 2; do for l in ${LIBS:-base cur}; do
  lib=$PWD/abl/$l.so; [ "$l" = cur ] && lib=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so
  KPLACE_LIB=$lib timeout -k 10 180 python3 tools/stream_time.py >> $OUT/st.txt 2>&1 || { tail -5 $OUT/st.txt; exit 1; }
done; done
cat $OUT/st.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for l in ${LIBS:-base cur}; do
  lib=$PWD/abl/$l.so; [ "$l" = cur ] && lib=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/libkplace.so
  BATCHES=30 KPLACE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_$l -o run -- python3 tools/stream_time.py > $OUT/ks_$l.log 2>&1 || exit $?
  rm -f $OUT/ks_$l/run_kernel_trace.csv
  python3 -c "
import csv,re
rows=sorted(csv.DictReader(open('$OUT/ks_$l/run_kernel_stats.csv')),key=lambda r:-float(r['TotalDurationNs']))
print('== $l')
for r in rows[:10]:
    m=re.search(r'(k_\w+|rocprim\w*|__amd\w+)',r['Name']); k=m.group(0) if m else r['Name'][:30]
    print(f'  {float(r[\"TotalDurationNs\"])/30/1e3:9.1f} us/batch {int(r[\"Calls\"])/30:7.1f} calls  avg {float(r[\"AverageNs\"])/1e3:7.2f} us  {k}')
"
done
