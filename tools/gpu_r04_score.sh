# r04: k_score32c (class form) parity + the score-matrix bench leg, and the FETCH/WRITE
# PMC of kp_score_dev (config #3 full queue).
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -m gpu -x -q -k "score or fused or materialised or abi" --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_score.log 2>&1 || { tail -30 gpurun_out/r04/pytest_score.log; exit 1; }
tail -1 gpurun_out/r04/pytest_score.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --out gpurun_out/r04/bench_score.json > gpurun_out/r04/bench_score.log 2>&1 || { tail -20 gpurun_out/r04/bench_score.log; exit 1; }
python3 -c "import json;b=json.load(open('gpurun_out/r04/bench_score.json'));print(json.dumps(b['score_matrix'],indent=1))"
