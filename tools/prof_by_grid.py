"""Per (kernel, grid size) launch statistics from a rocprofv3 --kernel-trace CSV: the bench
launch of k_relax (8192 workgroups) separated from the smaller probe / frontier launches.

    python tools/prof_by_grid.py gpurun_out/<tag>_stats/run_kernel_trace.csv > profiles/<tag>_kernel_summary.txt"""
import collections
import csv
import sys


def main(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        acc[(name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(f"# {path}\n# kernel, workgroups, launches, avg ms, min ms, max ms")
    for (name, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name:60s} {g:8d} {len(v):5d} {sum(v) / len(v):10.4f} {min(v):10.4f} {max(v):10.4f}")


if __name__ == "__main__":
    main(sys.argv[1])
