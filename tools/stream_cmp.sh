set -o pipefail
timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --stream-jobs 200000 --out gpurun_out/s_thr.json > gpurun_out/s_thr.log 2>&1 || exit $?
KP_SELECT_GENERIC=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --stream-jobs 200000 --out gpurun_out/s_gen.json > gpurun_out/s_gen.log 2>&1 || exit $?
timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -q -m gpu -k "wide or streaming" > gpurun_out/s_test.log 2>&1; echo rc=$?
