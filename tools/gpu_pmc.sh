# HBM traffic of the filter+score kernel: FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (TCC slots: FETCH_SIZE uses 3, WRITE_SIZE 2), kernel trace only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'k_score|k_select' --output-format csv \
    -d gpurun_out/pmc/$C -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream \
    > gpurun_out/pmc/$C.log 2>&1 || exit $?
  echo "$C ok"
done
