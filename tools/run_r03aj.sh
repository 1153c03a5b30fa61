#!/bin/bash
# r03: wino9_x6 next-tile patch in six 4-row parts (two in flight) vs three 8-row parts (library form).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "" _p6; do
    echo "== wino9_x6_bench$v"
    timeout -k 10 60 tools/wino9_x6_bench$v 1 | grep "wino9_x6 B\|max |"
    rc=$?; [ $rc -ge 124 ] && { echo "TIMEOUT/KILL $rc"; exit 1; }
  done
done > gpurun_out/w9_p6.log 2>&1
cat gpurun_out/w9_p6.log
