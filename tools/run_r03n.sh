#!/bin/bash
# r03: conv_bf3 MFMA-row -> pixel remap (conflict-free halo reads) against row-major, VGG layers at B=4;
# then the wino9_x6 channel-16 b64 A/B (run_r03m.sh).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in rowmajor remap rowmajor remap; do
    echo "== $v" >> gpurun_out/bf3remap.log
    timeout -k 5 120 tools/conv_bench_$v 4 vgg >> gpurun_out/bf3remap.log 2>&1 || { tail -20 gpurun_out/bf3remap.log; exit 1; }
done
cat gpurun_out/bf3remap.log
bash tools/run_r03m.sh
