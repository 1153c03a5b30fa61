#!/bin/bash
# round 5: wino9f3 standalone (timing, accuracy vs wino9 f32) and its per-unit phase timeline with the skip knobs
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for b in wino9f3_bench wino9f3_bench_prof wino9f3_bench_skip1 wino9f3_bench_skip2 wino9f3_bench_skip4 wino9f3_bench_skip8; do
  echo "== $b" >> gpurun_out/f3_r05e.log
  timeout -k 10 120 tools/$b 1 >> gpurun_out/f3_r05e.log 2>&1 || { tail -20 gpurun_out/f3_r05e.log; exit 1; }
done
cat gpurun_out/f3_r05e.log
