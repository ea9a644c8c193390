#!/usr/bin/env python3
"""Turn a gpurun_out/prof_<tag>/ rocprofv3 run into committed evidence under profiles/<tag>/.

    python scripts/summarize_profile.py r01

Writes
  profiles/<tag>/kernel_stats.csv      rocprofv3 --kernel-trace --stats summary (same bench command)
  profiles/<tag>/pmc_combine.json      FETCH_SIZE / WRITE_SIZE per combine launch (separate passes)
  profiles/<tag>/bench_traced.json     the bench JSON line printed under the tracer
  profiles/combine_traffic.json        HBM bytes per combine launch per (rows, dim), read by bench.py ("traffic")
HBM bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024: rocprofv3 reports both in KiB, and on gfx950
FETCH_SIZE counts exactly half of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM).
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pmc_values(path, counter, kernel_substr):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and kernel_substr in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return vals


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench_traced.json"), os.path.join(dst, "bench_traced.json"))
    bench = json.loads(open(os.path.join(src, "bench_traced.json")).read().strip().splitlines()[-1])
    rows, dim = bench["config"]["participations_per_gpu"], bench["config"]["dim"]
    tile = bench["config"].get("tile_rows")
    rows = tile or rows

    fetch = pmc_values(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE",
                       "combine_exact_kernel")
    write = pmc_values(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE",
                       "combine_exact_kernel")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    hbm = 2 * f_kib * 1024 + w_kib * 1024
    algo = 8.0 * rows * dim + (16.0 if tile else 8.0) * dim      # a tile launch also reads its partial
    # the headline launches: combine dispatches of the rows x dim matrix (the codec leg's smaller
    # combines share the kernel; they are the short ones and are left out)
    with open(os.path.join(src, "trace", "run_kernel_trace.csv")) as f:
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(f)
                if "combine_exact_kernel" in r["Kernel_Name"]]
    head = [d for d in durs if d >= 0.5 * max(durs)]
    comb = {"AverageNs": statistics.fmean(head), "Calls": len(head)}
    pmc = {"kernel": "combine_exact_kernel", "rows": rows, "dim": dim, "launches": len(fetch),
           "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib,
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": algo, "traffic_over_algorithmic": hbm / algo,
           "trace_avg_ns": float(comb["AverageNs"]), "trace_calls": int(comb["Calls"]),
           "bench_live_kernel_ms": bench["kernel_ms"],
           "note": "FETCH_SIZE doubled (gfx950 counts half of wide streaming reads); separate --pmc passes"}
    with open(os.path.join(dst, "pmc_combine.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    path = os.path.join(ROOT, "profiles", "combine_traffic.json")
    try:
        launches = json.load(open(path))["launches"]
    except (OSError, ValueError, KeyError):
        launches = []
    launches = [t for t in launches if (t.get("rows"), t.get("dim")) != (rows, dim)]
    launches.append({"rows": rows, "dim": dim, "hbm_bytes_per_launch": hbm, "source": f"profiles/{tag}/pmc_combine.json"})
    with open(path, "w") as f:
        json.dump({"launches": launches}, f, indent=1)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
