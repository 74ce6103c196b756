"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace CSV.

    python tools/prof_summary.py profiles/r01_stats/run_kernel_trace.csv

bench.py launches k_relax once on a 1024-node probe (incumbent = DOUBLE_MIN) before the
timed steps; grouping by grid size separates it from the bench launches (grid = nodes
per GPU x 64 lanes)."""
import csv
import sys
from collections import defaultdict


def main(path):
    groups = defaultdict(list)
    with open(path) as fh:
        for row in csv.DictReader(fh):
            name = row["Kernel_Name"]
            if "rocclr" in name:
                continue
            short = name.split("(")[0].replace("void ", "")
            groups[(short, int(row["Grid_Size_X"]), int(row["LDS_Block_Size"]), int(row["VGPR_Count"]),
                    int(row["Accum_VGPR_Count"]), int(row["Scratch_Size"]))].append(
                (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    print(f"{'kernel':28s} {'grid':>8s} {'lds':>6s} {'vgpr':>5s} {'agpr':>5s} {'scr':>4s} {'calls':>5s} "
          f"{'avg_ms':>10s} {'min_ms':>10s} {'max_ms':>10s}")
    for (k, g, lds, v, a, s), d in sorted(groups.items()):
        print(f"{k:28s} {g:8d} {lds:6d} {v:5d} {a:5d} {s:4d} {len(d):5d} {sum(d) / len(d):10.4f} {min(d):10.4f} {max(d):10.4f}")


if __name__ == "__main__":
    main(sys.argv[1])
