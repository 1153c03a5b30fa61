#!/bin/bash
# round 5: conv_lite single-chunk x6 layers with two staged register sets (LITE_NSET2_X6) vs one, standalone
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2; do for b in lite_bench_x6 lite_bench_x6n2; do
  echo "== $b" >> gpurun_out/lite_n2_r05ae.log
  timeout -k 10 120 tools/$b 100 >> gpurun_out/lite_n2_r05ae.log 2>&1 || exit 1
done; done
grep -E "==|B=1 .* us " gpurun_out/lite_n2_r05ae.log
