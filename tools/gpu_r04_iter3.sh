# r04: full -m gpu suite on the in-tree build, then A/B of builds (config #3 + #4).
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu3.log 2>&1
rc=$?
tail -2 gpurun_out/r04/pytest_gpu3.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" gpurun_out/r04/pytest_gpu3.log | head -30; exit $rc; }
C4=1 bash tools/ab_libs.sh
