cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/trstream; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-config4 --place-steps 0 --stream-jobs 100000 --no-kernel-events > $OUT/bench.log 2>&1
echo rc=$?
