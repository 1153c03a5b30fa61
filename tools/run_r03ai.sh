#!/bin/bash
# r03: wino_x6 knob removal incl. the per-chunk barrier (bit 3): base, no barrier (8), no U/transform/staging (7),
# and that without the barrier (15). Knob builds compute wrong results by construction; times only.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _s8 _s7 _s15; do
    echo "== wino_x6_bench$v"
    timeout -k 10 60 tools/wino_x6_bench$v 1 128 1 | grep "wino_x6 B"
    rc=$?; [ $rc -ge 124 ] && { echo "TIMEOUT/KILL $rc"; exit 1; }
  done
done > gpurun_out/x6_barrier.log 2>&1
cat gpurun_out/x6_barrier.log
