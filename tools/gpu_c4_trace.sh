# Kernel trace of config #4 solves (tools/c4_time.py), summarised per pass
# by tools/pass_trace_sum.py on the box (the raw trace stays there).
set -o pipefail
mkdir -p gpurun_out/c4t${SUFFIX}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4t${SUFFIX} -o run -- python3 tools/c4_time.py > gpurun_out/c4t${SUFFIX}/run.log 2>&1 || exit 1
python3 tools/pass_trace_sum.py gpurun_out/c4t${SUFFIX}/run_kernel_trace.csv > gpurun_out/c4t${SUFFIX}/pass_sum.txt && python3 tools/round_kernel_sum.py gpurun_out/c4t${SUFFIX}/run_kernel_trace.csv > gpurun_out/c4t${SUFFIX}/round_sum.txt
rm -f gpurun_out/c4t${SUFFIX}/run_kernel_trace.csv
cat gpurun_out/c4t${SUFFIX}/pass_sum.txt | head -30
