# score launch geometry sweep (bench with kernel events; roofline avg launch)
set -o pipefail
mkdir -p gpurun_out/sweep
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for npl in 2 4; do
  KP_SCORE_NPL=$npl timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --no-kernel-events --out gpurun_out/sweep/n_$npl.json > /dev/null 2>&1 || exit $?
  KP_SCORE_NPL=$npl timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream --out gpurun_out/sweep/e_$npl.json > /dev/null 2>&1 || exit $?
  python3 -c "import json;b=json.load(open('gpurun_out/sweep/n_$npl.json'));e=json.load(open('gpurun_out/sweep/e_$npl.json'));t=e['roofline'];print('npl $npl', round(b['ms_per_step'],2),'ms (events', round(e['ms_per_step'],2),') frac',round(t['frac'],3),'avg us',round(t['avg_launch_ms']*1e3,1))"
done
