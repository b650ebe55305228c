#!/usr/bin/env python3
"""rocprofv3 kernel trace vs bench.py's own event timing over the timed region.

Usage: python3 tools/rocprof_timed_region.py TRACE_CSV BENCH_JSON KERNEL_SUBSTR [command text]
Run the bench under `rocprofv3 --kernel-trace --stats` with --latency-searches 0 --http-requests 0
--no-cpu-baseline, so its timed launches are the trace's last `roofline.launches` dispatches of the
kernel; prints the average dispatch duration of those against the bench's HIP-event average.
"""
import csv
import json
import sys


def main():
    trace, bench, kern = sys.argv[1:4]
    cmd = sys.argv[4] if len(sys.argv) > 4 else ""
    rows = [r for r in csv.DictReader(open(trace)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    b = json.loads(open(bench).read().strip().splitlines()[-1])
    n = b["roofline"]["launches"]
    timed = dur[-n:]
    avg = sum(timed) / len(timed)
    name = rows[0]["Kernel_Name"].split("(")[0].replace("void ", "").replace("npow::", "")
    ev = b["roofline"]["avg_launch_ms"]
    print(f"rocprofv3 --kernel-trace --stats -- {cmd}")
    print()
    print(f"{name} dispatches in the whole run: {len(dur)} (warmup {len(dur) - n} + timed {n}), "
          f"average {sum(dur) / len(dur):.4f} ms")
    print(f"timed region = the last {n} dispatches (the bench's own launch count): average {avg:.4f} ms, "
          f"min {min(timed):.4f}, max {max(timed):.4f}")
    print(f"bench.py under the profiler, HIP events on the kernel's stream: avg_launch_ms {ev} over {n} launches "
          f"-> agreement {abs(avg - ev) / ev * 100:.2f} %")
    print(f"bench under the profiler: value {b['value']} Gnonce/s, kernel_gnps {b['roofline']['kernel_gnps']}, "
          f"frac {b['roofline']['frac']}, in-kernel clock {b['sclk_mhz']['mean']} MHz")


if __name__ == "__main__":
    main()
