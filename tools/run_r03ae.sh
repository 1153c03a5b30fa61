#!/bin/bash
# r03: wino9_x6 knob-removal timings: base, no next-tile patch loads (16), no U loads (1), both (17),
# no transform + no split (10). Outputs of the knob builds are wrong by construction; only the times matter.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _s16 _s1 _s17 _s10; do
    echo "== wino9_x6_bench$v"
    timeout -k 10 60 tools/wino9_x6_bench$v 1 | grep "wino9_x6 B"
    rc=$?; [ $rc -ge 124 ] && { echo "TIMEOUT/KILL $rc"; exit 1; }
  done
done > gpurun_out/w9_skip.log 2>&1
cat gpurun_out/w9_skip.log
