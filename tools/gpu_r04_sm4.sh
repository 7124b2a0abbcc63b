# r04: kernel durations of kp_score_dev (rocprofv3 --stats): full, scores only, mask only
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sm4
for v in full no-mask no-score; do
  a=; [ $v != full ] && a=--$v
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sm4/$v -o run -- python3 tools/score_dev_time.py $a > gpurun_out/sm4/$v.log 2>&1 || exit $?
  cat gpurun_out/sm4/$v.log
  rm -f gpurun_out/sm4/$v/run_kernel_trace.csv
done
python3 tools/kstats_cmp.py gpurun_out/sm4/full/run_kernel_stats.csv gpurun_out/sm4/no-mask/run_kernel_stats.csv gpurun_out/sm4/no-score/run_kernel_stats.csv
