#!/bin/bash
# r03: wino9_x6 next-tile patch loads: cache policy (nt / sc0) and issue point (after the MFMAs) vs the library form
# and the no-patch-load bound (knob 16).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _nt _sc0 _late _s16; do
    echo "== wino9_x6_bench$v"
    timeout -k 10 60 tools/wino9_x6_bench$v 1 | grep "wino9_x6 B\|max |"
    rc=$?; [ $rc -ge 124 ] && { echo "TIMEOUT/KILL $rc"; exit 1; }
  done
done > gpurun_out/w9_patch.log 2>&1
cat gpurun_out/w9_patch.log
