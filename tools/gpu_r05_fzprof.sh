# r05: k_score_topk phase clocks (abl/fzprof.so = the tree built with
# -DKP_FZ_PROFILE; KP_FZ_PROF=1): per-phase s_memtime sums over all waves,
# config #3 (6 solves) and config #4 (3 solves).
set -o pipefail
OUT=gpurun_out/r05fzp; rm -rf $OUT; mkdir -p $OUT
export KP_DEBUG_KNOBS=1 KP_FZ_PROF=1 KPLACE_LIB=$PWD/abl/fzprof.so
timeout -k 10 120 python3 tools/cfg_time.py > $OUT/c3.txt 2>&1 || { cat $OUT/c3.txt; exit 1; }
timeout -k 10 180 python3 tools/c4_time.py > $OUT/c4.txt 2>&1 || { cat $OUT/c4.txt; exit 1; }
grep -h "kp_fz_prof\|solve ms" $OUT/c3.txt $OUT/c4.txt
