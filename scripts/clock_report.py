#!/usr/bin/env python3
"""Per-dispatch shader clock from scripts/clock_pass.sh: GRBM_GUI_ACTIVE (summed over the 8 XCDs, so
/ 8) over the dispatch's kernel-trace duration, per kernel, in launch order.

    python scripts/clock_report.py gpurun_out/clock_<tag> [min_grid]
"""
import collections
import csv
import os
import sys


def main():
    d = sys.argv[1]
    min_grid = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    cyc = collections.defaultdict(float)
    valu = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cyc[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        elif r["Counter_Name"] == "SQ_INSTS_VALU":
            valu[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        if g < min_grid:
            continue
        did = int(r["Dispatch_Id"])
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if did in cyc:
            per[name].append((ns / 1e3, cyc[did] / 8, cyc[did] / 8 / ns, valu[did]))
    for name, rows in per.items():
        print(name)
        print("   us        cycles      GHz   VALU/launch")
        for us, c, ghz, v in rows:
            print(f"   {us:8.1f}  {c:10.0f}  {ghz:5.2f}  {v:.3g}")
        us = sorted(x[0] for x in rows)
        print(f"   -> {len(rows)} launches: median {us[len(us)//2]:.1f} us, cycles median "
              f"{sorted(x[1] for x in rows)[len(rows)//2]:.0f}, clock {min(x[2] for x in rows):.2f}-{max(x[2] for x in rows):.2f} GHz")


if __name__ == "__main__":
    main()
