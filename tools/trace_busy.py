"""Busy time per kernel and GPU idle share of a rocprofv3 --kernel-trace CSV (all kernels
of one stream-serial program): sum of durations by kernel, the union of busy intervals over
the traced span, and the gaps between consecutive kernels.

    python tools/trace_busy.py gpurun_out/<dir>/run_kernel_trace.csv [t_from_s]"""
import csv
import sys
from collections import defaultdict


def main(path, t_from=0.0):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
    rows.sort()
    t0 = rows[0][0]
    rows = [r for r in rows if r[0] - t0 >= t_from * 1e9]
    by = defaultdict(lambda: [0, 0.0])
    busy, cur_s, cur_e = 0, None, None
    for s, e, k in rows:
        by[k][0] += 1
        by[k][1] += (e - s) / 1e6
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    print(f"span {span / 1e9:.3f} s, busy {busy / 1e9:.3f} s ({busy / span:.1%}), kernels {len(rows)}")
    for k, (n, ms) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:40s} {n:7d} calls {ms:10.1f} ms  {ms / (span / 1e6):6.1%}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
