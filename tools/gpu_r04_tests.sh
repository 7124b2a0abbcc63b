# r04: the full GPU suite on the working tree
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r04/pytest.log
exit $rc
