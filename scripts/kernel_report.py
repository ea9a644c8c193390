#!/usr/bin/env python3
"""Per-kernel counter report from one round's rocprofv3 runs (trace stats + PMC passes).

    python scripts/kernel_report.py gpurun_out/prof_<tag>/trace gpurun_out/pmc_<tag>_shamir [...]

For every kernel seen in the PMC directories: average dispatch duration (kernel-trace stats),
SQ_INSTS_VALU per launch and per wave, lane-ops/s = SQ_INSTS_VALU x 64 / duration, the VALU issue
share SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (both in quad-cycles), and HBM bytes per launch
(2 x FETCH_SIZE + WRITE_SIZE, KiB; FETCH_SIZE doubled on gfx950, MI355X_MICROARCH.md HBM).
Prints JSON keyed by the short kernel name.
"""
import collections
import csv
import glob
import json
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    trace, pmcs = sys.argv[1], sys.argv[2:]
    dur = {}
    for f in glob.glob(trace + "/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Name"])] = (float(r["AverageNs"]), int(r["Calls"]), float(r["MinNs"]), float(r["MaxNs"]))
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in pmcs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        c = {n: max(v) for n, v in cs.items()}          # the largest dispatch of the kernel: the bench launch
        rec = {"counters_max_dispatch": c}
        if k in dur:
            rec["trace_avg_ns"], rec["trace_calls"], rec["trace_min_ns"], rec["trace_max_ns"] = dur[k]
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c and c["SQ_WAVES"]:
            rec["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / c["SQ_WAVES"]
        if "SQ_ACTIVE_INST_VALU" in c and c.get("SQ_WAVE_CYCLES"):
            rec["valu_active_per_wave_cycle"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rec["hbm_bytes"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        out[k] = rec
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
