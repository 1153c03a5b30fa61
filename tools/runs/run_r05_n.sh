#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2; do for b in wino_x6_bench_prof0 wino_x6_bench_prof; do
  echo "== $b" >> gpurun_out/x6args_r05n.log
  timeout -k 10 120 tools/$b 1 128 1 0 0 0 0 1 1 >> gpurun_out/x6args_r05n.log 2>&1 || exit 1
done; done
grep -E "==|issue split|timeline|wino_x6 B" gpurun_out/x6args_r05n.log
