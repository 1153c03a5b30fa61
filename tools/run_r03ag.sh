#!/bin/bash
# r03: wino9_x6 with the next tile's patch / U loads unconditional (library form now) vs the branch form (_cond)
# and the no-patch-load bound (_s16).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _cond _s16; do
    echo "== wino9_x6_bench$v"
    timeout -k 10 60 tools/wino9_x6_bench$v 1 | grep "wino9_x6 B\|max |"
    rc=$?; [ $rc -ge 124 ] && { echo "TIMEOUT/KILL $rc"; exit 1; }
  done
done > gpurun_out/w9_uncond.log 2>&1
cat gpurun_out/w9_uncond.log
