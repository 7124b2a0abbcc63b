set -o pipefail
mkdir -p gpurun_out/prof1
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1/bench.log 2>&1
echo "rocprof rc=$?"
ls -R gpurun_out/prof1 | head -20
