#!/usr/bin/env python3
"""Recompute bench.py's `roofline.frac` from a committed rocprofv3 kernel summary.

bench.py times the dominant kernel inside the headline's hipGraph frame replay (bench.graph_layer_ms: in-kernel end
stamps, a layer's share = its end minus its predecessor's end); rocprofv3 --kernel-trace times every launch on the
device. This script takes the executed FLOPs per launch that bench reports for the dominant kernel, divides by
rocprof's average duration of the same kernel (all template instantiations that share bench's short name,
launch-weighted) and compares the resulting fraction of the pipe's peak with bench's own.

With a kernel TRACE (run_kernel_trace.csv) only the graph-replayed frames count: the dispatches are grouped into
frames at each launch of the frame's first kernel (the start conv), and a frame is a graph
replay when its kernels ran back to back (span - sum of durations < 5 us; eager frames have host launch gaps). With a
kernel STATS file every launch counts (graph and eager alike).

Usage: python tools/roofline_check.py <bench_json_line_file> <kernel_trace.csv | kernel_stats.csv> [tolerance=0.02]
Exit status 1 when the two fractions differ by more than the tolerance (relative).
"""
import csv
import gzip
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


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def trace_graph_avg_ns(path, name, frame_start="wino9f3_"):
    rows = sorted(csv.DictReader(_open(path)), key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], None
    for r in rows:
        if frame_start in r["Kernel_Name"] and "<true>" not in r["Kernel_Name"]:
            cur = []
            frames.append(cur)
        if cur is not None:
            cur.append(r)
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])   # noqa: E731
    calls, total, nframes = 0, 0.0, 0
    for fr in frames:
        span = int(fr[-1]["End_Timestamp"]) - int(fr[0]["Start_Timestamp"])
        if span - sum(dur(r) for r in fr) >= 5000:
            continue   # an eager frame (host launch gaps between its kernels)
        nframes += 1
        for r in fr:
            if short_name(r["Kernel_Name"]) == name:
                calls += 1
                total += dur(r)
    return (total / calls if calls else None), calls, nframes


def main():
    b = bench_line(sys.argv[1])
    tol = float(sys.argv[3]) if len(sys.argv) > 3 else 0.02
    rf = b["roofline"]
    frames = None
    if "Start_Timestamp" in _open(sys.argv[2]).readline():
        avg_ns, calls, frames = trace_graph_avg_ns(sys.argv[2], rf["kernel"])
    else:
        avg_ns, calls = rocprof_avg_ns(sys.argv[2], rf["kernel"])
    if avg_ns is None:
        raise SystemExit(f"kernel {rf['kernel']!r} not in {sys.argv[2]}")
    achieved = rf["exec_flops_per_launch"] / (avg_ns * 1e-9) / 1e12
    frac = achieved / rf["peak"]
    rel = abs(frac - rf["frac"]) / rf["frac"]
    print(json.dumps({"kernel": rf["kernel"], "bench_avg_ms": rf["avg_launch_ms"], "rocprof_avg_ms": avg_ns * 1e-6,
                      "rocprof_calls": calls, "rocprof_graph_frames": frames, "bench_timing": rf.get("timing"),
                      "bench_frac": rf["frac"], "rocprof_frac": round(frac, 4),
                      "rel_diff": round(rel, 4), "within_tolerance": rel <= tol}))
    return 0 if rel <= tol else 1


if __name__ == "__main__":
    sys.exit(main())
