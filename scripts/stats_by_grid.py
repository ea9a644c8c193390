#!/usr/bin/env python3
"""rocprofv3 kernel-trace stats split by launch shape: the --stats summary averages every dispatch of
a kernel, mixing the bench's sizes (e.g. share-gen at 64 x 1M and at 10M-dim in the pipelines leg);
this groups the trace by (kernel, grid) instead.

    python scripts/stats_by_grid.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv > profiles/<tag>/kernel_stats_by_grid.csv
"""
import collections
import csv
import statistics
import sys


def main():
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        grid = (int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
        groups[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid_x", "grid_y", "grid_z", "calls", "avg_us", "median_us", "min_us", "max_us"])
    for (name, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, *grid, len(v), f"{statistics.fmean(v):.1f}", f"{statistics.median(v):.1f}",
                    f"{min(v):.1f}", f"{max(v):.1f}"])


if __name__ == "__main__":
    main()
