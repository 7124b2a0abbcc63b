# r04 baseline: kernel trace of one config #3 solve (per-round plan/accept), then the
# launch-floor probe (KP_HOST_PROF: no-op / dead-plan / dead-accept launches).
set -o pipefail
bash tools/gpu_trace.sh _r04a || exit 1
python3 tools/trace_rounds.py gpurun_out/trace_r04a/run_kernel_trace.csv --all > gpurun_out/trace_r04a/rounds.txt 2>&1
python3 tools/ktrace_sum.py gpurun_out/trace_r04a/run_kernel_trace.csv > gpurun_out/trace_r04a/sum.txt 2>&1
KP_DEBUG_KNOBS=1 KP_HOST_PROF=1 timeout -k 10 120 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > gpurun_out/trace_r04a/hostprof.log 2>&1
echo "hostprof rc=$?"
grep -h "kp_probe\|kp_host_prof" gpurun_out/trace_r04a/hostprof.log | tail -12
# per-pass in-kernel spans (KP_PASS_PROFILE build): plan span, accept span, gap
KPLACE_LIB=$PWD/ab/passprof.so KP_DEBUG_KNOBS=1 KP_FZ_PROF=1 KP_PASS_SPANS=1 timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events > gpurun_out/trace_r04a/spans.log 2>&1
echo "spans rc=$?"
grep -c kp_pass_span gpurun_out/trace_r04a/spans.log
