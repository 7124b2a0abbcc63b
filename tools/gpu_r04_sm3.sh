# r04: k_score32c with non-temporal score stores: score parity tests, timing, bench line
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "score or golden or knob" --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_sm.log 2>&1 || { tail -30 gpurun_out/r04/pytest_sm.log; exit 1; }
tail -1 gpurun_out/r04/pytest_sm.log
for i in 1 2; do timeout -k 10 120 python3 tools/score_dev_time.py || exit $?; done
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 > gpurun_out/r04/bench_nt.json 2> gpurun_out/r04/bench_nt.err || exit $?
python3 -c "import json;b=json.loads(open('gpurun_out/r04/bench_nt.json').read().strip().splitlines()[-1]);s=b['score_matrix'];print('bench', round(b['ms_per_step'],3), 'score_matrix', round(s['ms_per_call'],3), round(s['achieved']), round(s['frac'],3))"
