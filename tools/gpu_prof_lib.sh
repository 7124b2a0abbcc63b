# Kernel trace of the bench for one alternative library build ($1 = build/ab name).
set -o pipefail
LIB=$PWD/kubernetes-native-distributed-ai-job-scheduler_amd/build/ab/$1.so
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_$1; mkdir -p gpurun_out/prof_$1
KPLACE_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-kernel-events > gpurun_out/prof_$1/bench.log 2>&1
echo "rocprof rc=$?"
