#!/usr/bin/env python3
"""Recompute bench.py's `roofline.frac` from a committed rocprofv3 kernel-stats summary.

bench.py times the dominant kernel with HIP events on the forward's stream; rocprofv3 --kernel-trace
--stats times every launch on the device. This script takes the executed FLOPs per launch that bench
reports for the dominant kernel, divides by rocprof's average duration of the same kernel (all template
instantiations that share bench's short name, launch-weighted) and compares the resulting fraction of
the pipe's peak with bench's own.

Usage: python tools/roofline_check.py <bench_json_line_file> <kernel_stats.csv> [tolerance=0.05]
Exit status 1 when the two fractions differ by more than the tolerance (relative).
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short_name  # noqa: E402


def bench_line(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and '"roofline"' in line:
            return json.loads(line)
    raise SystemExit(f"{path}: no bench JSON line")


def rocprof_avg_ns(path, name):
    calls, total = 0, 0.0
    for r in csv.DictReader(open(path)):
        if short_name(r["Name"]) == name:
            calls += int(r["Calls"])
            total += float(r["TotalDurationNs"])
    return (total / calls if calls else None), calls


def main():
    b = bench_line(sys.argv[1])
    tol = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05
    rf = b["roofline"]
    avg_ns, calls = rocprof_avg_ns(sys.argv[2], rf["kernel"])
    if avg_ns is None:
        raise SystemExit(f"kernel {rf['kernel']!r} not in {sys.argv[2]}")
    achieved = rf["exec_flops_per_launch"] / (avg_ns * 1e-9) / 1e12
    frac = achieved / rf["peak"]
    rel = abs(frac - rf["frac"]) / rf["frac"]
    print(json.dumps({"kernel": rf["kernel"], "bench_avg_ms": rf["avg_launch_ms"], "rocprof_avg_ms": avg_ns * 1e-6,
                      "rocprof_calls": calls, "bench_frac": rf["frac"], "rocprof_frac": round(frac, 4),
                      "rel_diff": round(rel, 4), "within_tolerance": rel <= tol}))
    return 0 if rel <= tol else 1


if __name__ == "__main__":
    sys.exit(main())
