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
    # round 4: the roofline fraction recomputed from this profile alone (bench.py names this file in
    # roofline.profile when its build_sha16 equals the bench's own)
    ro = b["roofline"]
    npl = ro["nonces_per_launch"]
    ex = ro.get("executed_ops_per_nonce", 2086)
    peak = ro["peak"]
    frac = npl * ex / (avg * 1e-3) / 1e12 / peak
    print()
    if "build_sha16" in b:
        print(f"build_sha16 {b['build_sha16']}")
    print(f"nonces_per_launch {npl}")
    print(f"executed_ops_per_nonce {ex}")
    print(f"frac_executed_from_profile {frac:.4f}")
    print(f"  = {npl} nonces per launch x {ex} int32 ops / {avg:.4f} ms (the timed dispatches' rocprofv3 average) "
          f"/ {peak} Tops/s = {npl * ex / (avg * 1e-3) / 1e12:.3f} Tops/s / {peak}")
    if "frac_algorithmic" in ro:
        print(f"frac_algorithmic_from_profile {npl * 2232 / (avg * 1e-3) / 1e12 / peak:.4f} (2,232 ops per nonce)")
    # the box-independent figure: the fraction follows the box's power-limited clock (2,150-2,370 MHz by box),
    # the SIMD cycles per 64-nonce wave-hash do not (1,024 SIMDs x 64 lanes)
    mhz = b.get("sclk_mhz", {}).get("mean")
    if mhz:
        rate = npl / (avg * 1e-3)
        print(f"in_kernel_mhz {mhz}")
        print(f"cycles_per_hash_from_profile {1024 * 64 * mhz * 1e6 / rate:.1f}"
              f"  = 1,024 SIMDs x 64 lanes x {mhz} MHz / ({npl} nonces / {avg:.4f} ms)")


if __name__ == "__main__":
    main()
