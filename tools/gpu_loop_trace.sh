# kernel traces of one config #3 solve under knob settings: SETTINGS="A=1,B=2 C=3"
set -o pipefail
export KP_DEBUG_KNOBS=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for setting in $SETTINGS; do
  OUT=gpurun_out/ltrace$i; rm -rf $OUT; mkdir -p $OUT
  env ${setting//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 tools/cfg_time.py > $OUT/run.log 2>&1 || { echo "trace $setting failed"; exit 1; }
  f=$(find $OUT -name "*kernel_trace.csv" | head -1)
  echo "== $setting"; python3 tools/loop_trace.py $f > $OUT/rounds.txt && tail -25 $OUT/rounds.txt
  i=$((i+1))
done
