#!/bin/bash
# round 5: expand_0 in two 16-channel Cout blocks (conv_lite config 9) vs one 32-channel unit (RST_LITE_SPLIT=0):
# standalone times + output checks (accumulator and partials paths), timelines, then the transfer / layer tests
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=gpurun_out/lite_split_r05af.log
for sp in 0 1; do
  echo "== RST_LITE_SPLIT=$sp" >> $L
  RST_LITE_SPLIT=$sp timeout -k 10 120 tools/lite_bench_x6 100 >> $L 2>&1 || { tail -20 $L; exit 1; }
  RST_LITE_SPLIT=$sp LITE_PART=1 timeout -k 10 120 tools/lite_bench_x6 20 >> $L 2>&1 || { tail -20 $L; exit 1; }
  RST_LITE_SPLIT=$sp timeout -k 10 120 tools/lite_bench_x6prof 20 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
grep -E "==|expand_0|per step|per wave|MISMATCH" $L
TAG=r05af bash tools/gpu_measure.sh "tests=transfer or layer or expand or two_style or predictor" ab=RST_LITE_SPLIT=0@-@3
