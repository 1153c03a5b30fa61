#!/bin/bash
# round 5: wino9f3 with the half-unit tail launch: standalone timeline, start-conv parity, headline
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for b in wino9f3_bench wino9f3_bench_prof wino9f3_bench_skip1 wino9f3_bench_skip2; do
  echo "== $b" >> gpurun_out/f3_r05g.log
  timeout -k 10 120 tools/$b 1 >> gpurun_out/f3_r05g.log 2>&1 || { tail -20 gpurun_out/f3_r05g.log; exit 1; }
done
cat gpurun_out/f3_r05g.log
TAG=r05g bash tools/gpu_measure.sh "tests=start_conv_f3 or winograd_residual or winograd_full" short
