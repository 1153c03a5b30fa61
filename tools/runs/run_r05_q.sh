#!/bin/bash
# round 5: wino_x6 kernel arguments loaded in one batch (X6_ARGS_FIRST) vs the committed tree, same box; narrow-layer
# standalone timelines (x6 forms)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/lite_bench_x6 100 > gpurun_out/lite_r05q.log 2>&1 && timeout -k 10 120 tools/lite_bench_x6prof 20 >> gpurun_out/lite_r05q.log 2>&1 || { tail gpurun_out/lite_r05q.log; exit 1; }
cat gpurun_out/lite_r05q.log
TAG=r05q bash tools/gpu_measure.sh ab=RST_LIB=tools/librst_base.so@-@4
