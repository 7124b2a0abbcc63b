"""Summarise a rocprofv3 --stats kernel_stats.csv (one line per kernel)."""
import csv
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"void |kp::|\(anonymous namespace\)::|rocprim::ROCPRIM_\w+::detail::", "", name)
    head = name.split("(")[0]
    return head[:70]


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    tot = sum(int(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':70s} {'calls':>6} {'total ms':>9} {'avg us':>9} {'%':>6}")
    for r in rows:
        print(f"{short(r['Name']):70s} {int(r['Calls']):6d} {int(r['TotalDurationNs'])/1e6:9.2f} "
              f"{float(r['AverageNs'])/1e3:9.2f} {100*int(r['TotalDurationNs'])/tot:6.2f}")
    print(f"{'TOTAL':70s} {'':6s} {tot/1e6:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
