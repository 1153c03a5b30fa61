#!/bin/bash
# r03: wino9_x6 channel-16 reads as ds_read_b64 (v3) against b32 (v3a), alternating, standalone B=1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/w9ab.log
for i in 1 2 3; do
    for v in v3a v3; do
        echo "== $v $i" >> gpurun_out/w9ab.log
        timeout -k 5 60 tools/wino9_x6_bench_$v 1 >> gpurun_out/w9ab.log 2>&1
        rc=$?; if [ $rc -ge 124 ]; then tail -20 gpurun_out/w9ab.log; exit 1; fi
    done
done
grep -v "^\s*$" gpurun_out/w9ab.log | grep "==\|us" | head -40
