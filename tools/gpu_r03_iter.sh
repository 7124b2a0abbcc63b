# round-3 development iteration: parity suite (narrowed by PYTEST_PATHS), then
# config #3 solve timings of knob settings (tools/cfg_time.py, median of 5)
set -o pipefail
mkdir -p gpurun_out
PYTEST_PATHS="${PYTEST_PATHS:-tests/test_gpu_parity.py}" bash tools/gpu_test.sh || exit 1
for setting in ${SETTINGS:-"KP_PASS_LOOP=1"}; do
  env KP_DEBUG_KNOBS=1 ${setting//,/ } timeout -k 10 120 python tools/cfg_time.py >> gpurun_out/cfg_time.txt 2>&1 || { echo "cfg_time failed: $setting"; tail -5 gpurun_out/cfg_time.txt; exit 1; }
  echo "$setting: $(tail -1 gpurun_out/cfg_time.txt)"
done
