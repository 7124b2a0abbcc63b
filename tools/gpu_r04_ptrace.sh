# r04: per-pass plan / accept durations of one config #3 solve (rocprofv3
# kernel trace, tools/pass_trace_sum.py) for the in-tree build and ab/base.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pt
for lib in lib ab/base.so; do
  if [ "$lib" = lib ]; then n=lib; L=; else n=base; L=$PWD/$lib; fi
  KPLACE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pt/$n -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-stream --no-config4 --place-steps 0 --no-kernel-events --no-score-matrix --out gpurun_out/pt/$n.json > gpurun_out/pt/$n.log 2>&1 || exit $?
  python3 tools/pass_trace_sum.py gpurun_out/pt/$n/run_kernel_trace.csv > gpurun_out/pt/$n.sum.txt || exit $?
  python3 - gpurun_out/pt/$n/run_kernel_trace.csv > gpurun_out/pt/$n.gaps.txt <<'PY' || exit $?
import csv, sys, re
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_reset_units" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
tot = {}
for a, b in zip(seq, seq[1:]):
    k = re.sub(r"<.*", "", a["Kernel_Name"].replace("(anonymous namespace)", "")).split("::")[-1][:20] + " -> " + re.sub(r"<.*", "", b["Kernel_Name"].replace("(anonymous namespace)", "")).split("::")[-1][:20]
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    c, s = tot.get(k, (0, 0.0)); tot[k] = (c + 1, s + g)
dur = {}
for r in seq:
    k = re.sub(r"<.*", "", r["Kernel_Name"].replace("(anonymous namespace)", "")).split("::")[-1][:24]
    c, s = dur.get(k, (0, 0.0)); dur[k] = (c + 1, s + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"last solve span {span:.0f} us; kernels {sum(s for c, s in dur.values()):.0f} us; gaps {sum(s for c, s in tot.values()):.0f} us")
for k, (c, s) in sorted(dur.items(), key=lambda x: -x[1][1])[:10]:
    print(f"  kernel {k:26s} {c:5d} {s:9.0f} us avg {s / c:7.2f}")
for k, (c, s) in sorted(tot.items(), key=lambda x: -x[1][1])[:10]:
    print(f"  gap {k:46s} {c:5d} {s:9.0f} us avg {s / c:7.2f}")
PY
  rm -f gpurun_out/pt/$n/run_kernel_trace.csv
  head -22 gpurun_out/pt/$n.gaps.txt
  head -24 gpurun_out/pt/$n.sum.txt
done
