#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/wino9f3_bench_prof 1 > gpurun_out/f3_r05i.log 2>&1; cat gpurun_out/f3_r05i.log
