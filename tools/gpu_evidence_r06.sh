set -o pipefail
ROUND=r06 SKIP_C4=1 bash tools/gpu_evidence.sh || exit 1
bash tools/gpu_c4_profile.sh > gpurun_out/evidence/c4_profile.log 2>&1 || { tail -5 gpurun_out/evidence/c4_profile.log; exit 1; }
echo c4 profile ok
SUFFIX=_ev bash tools/gpu_c4_trace.sh > gpurun_out/evidence/c4_trace.log 2>&1 || { tail -5 gpurun_out/evidence/c4_trace.log; exit 1; }
echo c4 trace ok
cp gpurun_out/c4_profile/summary.txt gpurun_out/evidence/summary/r06_c4_profile.txt
{ echo "# config #4 kernel trace of tools/c4_time.py (rocprofv3 --kernel-trace): per pass index, summed / largest k_accept and k_plan launch (tools/pass_trace_sum.py); then per-round kernel times (tools/round_kernel_sum.py)"
  cat gpurun_out/c4t_ev/pass_sum.txt; echo; cat gpurun_out/c4t_ev/round_sum.txt; } > gpurun_out/evidence/summary/r06_c4_pass_trace.txt
