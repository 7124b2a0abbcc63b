# r06: RCCL API trace of the one-rank RCCL solve, config #3 per-round pass
# costs, and the default bench line (with the config #2 leg)
set -o pipefail
OUT=gpurun_out/r06b
rm -rf $OUT; mkdir -p $OUT/rccl $OUT/c3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --rccl-trace --kernel-trace --stats --output-format csv -d $OUT/rccl -o run -- python3 -m pytest tests/test_gpu_rccl.py -m gpu -x -q -k "rank_config3_full or rank_config4" > $OUT/rccl/pytest.log 2>&1 || { tail -30 $OUT/rccl/pytest.log; exit 1; }
tail -2 $OUT/rccl/pytest.log
ls $OUT/rccl
B3="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-score-matrix --no-phases --no-config2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/c3 -o run -- python3 $B3 > $OUT/c3/bench.log 2>&1 || { tail -20 $OUT/c3/bench.log; exit 1; }
python3 tools/c3_round_passes.py $OUT/c3/run_kernel_trace.csv > $OUT/c3/round_passes.txt && tail -8 $OUT/c3/round_passes.txt
rm -f $OUT/c3/run_kernel_trace.csv
timeout -k 10 600 python -u bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
python3 -c "import json;b=json.load(open('$OUT/bench.json'));print('solve', b['ms_per_step'], 'c2', json.dumps(b.get('config2'))[:600]); print('c4cpu', json.dumps(b['config4']['cpu_baseline'])[:1200])"
