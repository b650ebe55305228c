#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools/pmc_bench.sh) for one kernel into profiles/*.json.

Usage: python3 tools/pmc_summary.py <gpurun_out/pmc_TAG> <kernel-name substring> <what> <out.json>

Per dispatch of the kernel: FETCH_SIZE / WRITE_SIZE are kilobytes (rocprofv3 derived counters);
HBM bytes per launch = 2 x FETCH_SIZE (the gfx950 correction of MI355X_MICROARCH.md, an upper
bound for reads that are not 16-B/lane streams) + WRITE_SIZE, mean over the dispatches.
"""
import csv
import json
import os
import statistics
import sys


def load(path, kernel):
    per = {}  # (dispatch, counter) -> value
    for row in csv.DictReader(open(path)):
        if kernel not in row["Kernel_Name"]:
            continue
        key = (int(row["Dispatch_Id"]), row["Counter_Name"])
        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    by_counter = {}
    for (_, c), v in per.items():
        by_counter.setdefault(c, []).append(v)
    return by_counter


def main():
    base, kernel, what, out = sys.argv[1:5]
    counters = {}
    for sub in ("fetch", "write", "sq"):
        p = os.path.join(f"{base}_{sub}", "run_counter_collection.csv")
        if os.path.exists(p):
            counters.update(load(p, kernel))
    fetch, write = counters.get("FETCH_SIZE", []), counters.get("WRITE_SIZE", [])
    res = {
        "what": what,
        "kernel": kernel,
        "dispatches": len(fetch),
        "counters_median": {k: round(statistics.median(v), 4) for k, v in sorted(counters.items())},
        "counters_mean": {k: round(statistics.mean(v), 3) for k, v in sorted(counters.items())},
        "hbm_bytes_per_launch": (round((2 * statistics.mean(fetch) + statistics.mean(write)) * 1024)
                                 if fetch and write else None),
        "derivation": "FETCH_SIZE and WRITE_SIZE are kilobytes per dispatch (rocprofv3 derived counters); "
                      "FETCH doubled per the gfx950 correction (upper bound: these reads are not 16-B/lane "
                      "streams); mean over dispatches",
    }
    if "SQ_INSTS_VALU" in counters and "SQ_WAVES" in counters:
        res["valu_insts_per_wave"] = round(statistics.mean(counters["SQ_INSTS_VALU"]) /
                                           statistics.mean(counters["SQ_WAVES"]), 1)
    if "SQ_WAVE_CYCLES" in counters:
        wc = statistics.mean(counters["SQ_WAVE_CYCLES"])
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
            if c in counters:
                res[f"{c[3:].lower()}_frac_of_wave_cycles"] = round(statistics.mean(counters[c]) / wc, 4)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("dispatches", "hbm_bytes_per_launch")}))


if __name__ == "__main__":
    main()
