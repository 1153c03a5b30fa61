#!/bin/bash
# round 5: wino9f3 epilogue (transposed M image, buffer stores): standalone timeline, full GPU suite, smoke, bench, trace
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for b in wino9f3_bench_prof wino9f3_bench_skip1; do
  echo "== $b" >> gpurun_out/f3_r05k.log
  timeout -k 10 120 tools/$b 1 >> gpurun_out/f3_r05k.log 2>&1 || { tail -20 gpurun_out/f3_r05k.log; exit 1; }
done
cat gpurun_out/f3_r05k.log
TAG=r05k bash tools/gpu_measure.sh tests smoke bench prof
