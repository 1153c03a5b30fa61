#!/bin/bash
# r03: wino9_x6 with s_setprio 1 on one wave half (W9_SETPRIO 1 / 2) against the library form, standalone.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _p1 _p2; do
    echo "== wino9_x6_bench$v"
    timeout -k 10 60 tools/wino9_x6_bench$v 1 || { echo FAILED; exit 1; }
  done
done > gpurun_out/w9_setprio.log 2>&1 || { cat gpurun_out/w9_setprio.log; exit 1; }
grep -E "==|wino9_x6 B" gpurun_out/w9_setprio.log
