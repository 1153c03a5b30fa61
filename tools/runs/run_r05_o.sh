#!/bin/bash
# round 5: wino9f3 with the first U blocks of each MFMA phase prefetched before the transform: timeline, parity, headline
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for b in wino9f3_bench_prof wino9f3_bench; do
  echo "== $b" >> gpurun_out/f3_r05o.log
  timeout -k 10 120 tools/$b 1 >> gpurun_out/f3_r05o.log 2>&1 || { tail -20 gpurun_out/f3_r05o.log; exit 1; }
done
cat gpurun_out/f3_r05o.log
TAG=r05o bash tools/gpu_measure.sh "tests=start_conv_f3 or winograd_residual" short
