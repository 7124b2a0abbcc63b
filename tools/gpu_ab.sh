# A/B: bench with eager launches vs round graphs, kernel events off and on.
set -o pipefail
mkdir -p gpurun_out
for mode in eager graph; do
  for ev in noev ev; do
    extra=""; [ $ev = noev ] && extra="--no-kernel-events"
    env_=""; [ $mode = eager ] && export KP_NO_GRAPH=1 || unset KP_NO_GRAPH
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stream $extra --out gpurun_out/ab_${mode}_$ev.json > gpurun_out/ab_${mode}_$ev.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import json
for m in ("eager","graph"):
  for e in ("noev","ev"):
    b=json.load(open(f"gpurun_out/ab_{m}_{e}.json"))
    print(m, e, round(b["ms_per_step"],3), "ms", b["config"]["rounds"], b["config"]["passes"], b["config"]["placed_jobs"], "roof", round(b["roofline"]["frac"],3))
PY
