#!/bin/bash
# r03 same-box A/B: the pre-accumulator build (commit 2b12e2c, in _ab_old/) against HEAD, alternating short
# headline benches, then one kernel trace of each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --train-batch 0 --no-two-styles"
rm -f gpurun_out/ab.log
for i in 1 2 3; do
    (cd _ab_old && timeout -k 10 200 $B > ../gpurun_out/ab_old_$i.log 2>&1) || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
    timeout -k 10 200 $B > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
    echo "old $i: $(grep -o '"value": [0-9.]*' gpurun_out/ab_old_$i.log | head -1)   new $i: $(grep -o '"value": [0-9.]*' gpurun_out/ab_new_$i.log | head -1)" | tee -a gpurun_out/ab.log
done
(cd _ab_old && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/prof_ab_old -o run -- $B > ../gpurun_out/prof_ab_old.log 2>&1) || { tail -20 gpurun_out/prof_ab_old.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ab_new -o run -- $B > gpurun_out/prof_ab_new.log 2>&1 || { tail -20 gpurun_out/prof_ab_new.log; exit 1; }
ls gpurun_out/prof_ab_old gpurun_out/prof_ab_new
