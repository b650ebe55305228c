#!/usr/bin/env python3
"""Summary of a tools/pmc_dual_issue.sh pass: the per-dispatch median of each counter for the search kernel and the
dual-issue rate, SQ_ACTIVE_INST_VALU2 / (GRBM_GUI_ACTIVE x 32) -- the normalisation of profiles/r03s_pmc_dual_issue.json.

    python3 tools/pmc_dual_summary.py gpurun_out/pmc_dual_TAG/run_counter_collection.csv BUILD_SHA16 > out.json
"""
import csv
import json
import statistics
import sys

KERNEL = "npow_pool_kernel_ls2_arg<false>"


def main():
    path, sha = sys.argv[1], sys.argv[2]
    per = {}
    for row in csv.DictReader(open(path)):
        if KERNEL not in row["Kernel_Name"]:
            continue
        per.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
        per[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    med = {k: statistics.median(v.values()) for k, v in per.items()}
    out = {"what": "rocprofv3 --pmc SQ_ACTIVE_INST_VALU2 ... on python3 bench.py --no-cpu-baseline --steps 30 --warmup 3 "
                   "--latency-searches 0 --http-requests 0 --regime-searches 0 (tools/pmc_dual_issue.sh), build_sha16 "
                   + sha,
           "kernel": KERNEL, "dispatches": len(next(iter(per.values()))), "counters_median": med,
           "valu2_per_quad_cycle": round(med["SQ_ACTIVE_INST_VALU2"] / (med["GRBM_GUI_ACTIVE"] * 32), 4),
           "how": "valu2_per_quad_cycle = SQ_ACTIVE_INST_VALU2 / (GRBM_GUI_ACTIVE x 32), the normalisation of "
                  "r03s_pmc_dual_issue.json (0.580 there)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
