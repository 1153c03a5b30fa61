#!/bin/bash
# r03: same-box A/B of the VGG16 128-wide conv tile with / without the two-stage weight prefetch (RST_BF3_NO_WP2=1).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 12"
for i in 1 2 3; do
  timeout -k 10 400 $T > gpurun_out/bench_ab_on$i.log 2>&1 || { tail -30 gpurun_out/bench_ab_on$i.log; exit 1; }
  RST_BF3_NO_WP2=1 timeout -k 10 400 $T > gpurun_out/bench_ab_off$i.log 2>&1 || { tail -30 gpurun_out/bench_ab_off$i.log; exit 1; }
  echo "wp2: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ab_on$i.log | grep -o '"ms_per_step": [0-9.]*')   135: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ab_off$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
