# Round evidence in one GPU call (outputs under gpurun_out/evidence; summarise
# into profiles/ with tools/evidence_summary.py):
#   1. the full GPU test suite (SKIP_TESTS=1 skips)
#   2. the default bench line (SKIP_BENCH=1 skips)
#   3. rocprofv3 --kernel-trace --stats of the config #3 solve steps
#   4. the same for the config #4 (solve + preempt) and config #5 streaming legs
#   5. PMC passes (one counter group each): FETCH_SIZE, WRITE_SIZE, the SQ
#      issue/wait counters and the LDS bank-conflict counters of the hot kernels
#   6. a HIP runtime trace of kp_place calls (hipMalloc / hipFree inside steps)
#   7. config #4: per-kernel time and k_score_topk lane-ops per pair
#      (gpu_c4_profile.sh) and the per-pass kernel trace (gpu_c4_trace.sh)
set -o pipefail
OUT=gpurun_out/evidence
rm -rf $OUT; mkdir -p $OUT/prof $OUT/profsm $OUT/prof45 $OUT/pmc $OUT/rt
rocminfo 2>/dev/null | grep -m1 gfx950 > $OUT/arch.txt || true
if [ "$SKIP_TESTS" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
if [ "$SKIP_BENCH" != 1 ]; then
  timeout -k 10 600 python -u bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
  echo bench ok
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B3="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --no-config2 --place-steps 0 --no-score-matrix --no-phases"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $B3 --out $OUT/prof/bench_prof.json > $OUT/prof/bench.log 2>&1 || exit $?
echo prof ok
# the materialised score matrix + mask (kp_score_dev, config #3 full queue) on its own
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profsm -o run -- python3 tools/score_dev_time.py > $OUT/profsm/score_dev.log 2>&1 || exit $?
echo profsm ok
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof45 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-config2 --place-steps 0 --c4-steps 1 --no-phases --out $OUT/prof45/bench_prof.json > $OUT/prof45/bench.log 2>&1 || exit $?
echo prof45 ok
B1="bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stream --no-config4 --no-config2 --place-steps 0 --no-phases"
RE='k_score|k_select|k_merge|k_plan|k_accept'
pmc() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" --output-format csv \
    -d $OUT/pmc/$n -o run -- python3 $B1 > $OUT/pmc/$n.log 2>&1 || return $?
  echo "pmc $n ok"
}
pmc FETCH_SIZE FETCH_SIZE || exit $?
pmc WRITE_SIZE WRITE_SIZE || exit $?
pmc SQ1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
pmc LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES || exit $?
# the same SQ pass on a k_score_topk build without its select phase
# (ABOUT=$PWD/abl tools/build_variant.sh WORKTREE noselect -DKP_FZ_EXP=1): score + threshold
# stages alone; the select phase is the difference (its round 0 only: no
# candidates, the solve ends after one round)
NOSEL=${NOSEL:-abl/noselect.so}
if [ -f $NOSEL ]; then
  export KPLACE_LIB=$PWD/$NOSEL
  pmc SQ_NOSEL SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $?
  unset KPLACE_LIB
fi
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $OUT/rt -o run -- python3 tools/place_steps.py > $OUT/rt/place.log 2>&1 || exit $?
echo rt ok
# config #4: per-kernel time per solve + k_score_topk lane-ops per pair, and
# the per-pass / per-round kernel trace (SKIP_C4=1 skips)
if [ "$SKIP_C4" != 1 ]; then
  bash tools/gpu_c4_profile.sh > $OUT/c4_profile.log 2>&1 || { tail -5 $OUT/c4_profile.log; exit 1; }
  SUFFIX=_ev bash tools/gpu_c4_trace.sh > $OUT/c4_trace.log 2>&1 || { tail -5 $OUT/c4_trace.log; exit 1; }
  echo c4 ok
fi
python3 tools/evidence_summary.py ${ROUND:-r06} $OUT $OUT/summary && ls $OUT/summary
R=${ROUND:-r06}
if [ -f gpurun_out/c4_profile/summary.txt ]; then cp gpurun_out/c4_profile/summary.txt $OUT/summary/${R}_c4_profile.txt; fi
if [ -f gpurun_out/c4t_ev/pass_sum.txt ]; then
  { echo "# config #4 kernel trace of tools/c4_time.py (rocprofv3 --kernel-trace): per pass index, summed / largest k_accept and k_plan launch (tools/pass_trace_sum.py); then per-round kernel times (tools/round_kernel_sum.py)"
    cat gpurun_out/c4t_ev/pass_sum.txt; echo; cat gpurun_out/c4t_ev/round_sum.txt; } > $OUT/summary/${R}_c4_pass_trace.txt
fi
# the raw traces exceed what gpurun copies back: keep logs and summaries only
rm -f $OUT/prof/run_kernel_trace.csv $OUT/profsm/run_kernel_trace.csv $OUT/prof45/run_kernel_trace.csv $OUT/*/*/run_counter_collection.csv $OUT/*/*/run_kernel_trace.csv
du -sh $OUT
