# Config #4 kernel stats (3 solves of tools/c4_time.py) and the per-round
# changed-node / tile counts (tools/c4_rounds.py, first 40 rounds).
set -o pipefail
mkdir -p gpurun_out/c4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4/p4 -o run -- python3 tools/c4_time.py > gpurun_out/c4/p4.log 2>&1 || exit 1
rm -f gpurun_out/c4/p4/run_kernel_trace.csv
timeout -k 10 200 python -u tools/c4_rounds.py 40 > gpurun_out/c4/rounds.txt 2>&1 || exit 1
echo done
