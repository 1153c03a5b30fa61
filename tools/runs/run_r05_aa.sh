#!/bin/bash
# round 5: narrow-layer standalone times and per-step timelines (x6 forms)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/lite_bench_x6 100 > gpurun_out/lite_r05aa.log 2>&1 && timeout -k 10 120 tools/lite_bench_x6prof 20 >> gpurun_out/lite_r05aa.log 2>&1 || { tail -20 gpurun_out/lite_r05aa.log; exit 1; }
grep -v "^$" gpurun_out/lite_r05aa.log
