"""Side-by-side per-kernel totals of rocprofv3 --stats CSVs (analysis tool):
  python tools/kstats_cmp.py a/run_kernel_stats.csv b/run_kernel_stats.csv ...
Per kernel (template arguments stripped): calls and total ms in each file."""
import csv
import re
import sys


def load(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = re.sub(r"<.*", "", r["Name"].replace("(anonymous namespace)", "")).replace("void ", "").split("(")[0].split("::")[-1]
        c, t = out.get(name, (0, 0.0))
        out[name] = (c + int(r["Calls"]), t + float(r["TotalDurationNs"]) / 1e6)
    return out


def main():
    files = sys.argv[1:]
    tabs = [load(f) for f in files]
    names = sorted({k for t in tabs for k in t}, key=lambda k: -max(t.get(k, (0, 0))[1] for t in tabs))
    print("kernel".ljust(34) + "".join(f"{f.split('/')[-2][:18]:>26}" for f in files))
    for k in names[:24]:
        print(k[:33].ljust(34) + "".join(f"{t.get(k, (0, 0))[0]:>10d} {t.get(k, (0, 0))[1]:>10.3f} ms" for t in tabs))
    print("total".ljust(34) + "".join(f"{'':>10} {sum(v[1] for v in t.values()):>10.3f} ms" for t in tabs))


if __name__ == "__main__":
    main()
