"""Shrink a rocprofv3 --pmc counter_collection.csv to one row per (kernel, counter): the values
summed over the dispatches, the other columns from the first dispatch (bench.py's readers sum
per kernel and counter, so they read the same totals).  Usage: compact_pmc.py CSV [CSV ...]"""
import csv
import sys


def compact(path):
    with open(path) as fh:
        rows = list(csv.DictReader(fh))
    if not rows:
        return
    cols = list(rows[0].keys())
    acc, first, n = {}, {}, {}
    for r in rows:
        k = (r["Kernel_Name"], r["Counter_Name"])
        acc[k] = acc.get(k, 0.0) + float(r["Counter_Value"])
        n[k] = n.get(k, 0) + 1
        first.setdefault(k, r)
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=cols + ["Dispatches"])
        w.writeheader()
        for k, r in first.items():
            out = dict(r)
            out["Counter_Value"] = repr(acc[k])
            out["Dispatches"] = n[k]
            w.writerow(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        compact(p)
