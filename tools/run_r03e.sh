#!/bin/bash
# r03 experiment: frame time with the residual-conv finalizes skipped (upper bound of removing them; outputs wrong),
# and the kernel trace of the HEAD frame.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --train-batch 0 --no-ingest --pcie-steps 0 --no-two-styles"
timeout -k 10 200 $B > gpurun_out/e_base.log 2>&1 || { tail -30 gpurun_out/e_base.log; exit 1; }
RST_EXPERIMENT_SKIP_FIN=1 timeout -k 10 200 $B > gpurun_out/e_skip1.log 2>&1 || { tail -30 gpurun_out/e_skip1.log; exit 1; }
RST_EXPERIMENT_SKIP_FIN=2 timeout -k 10 200 $B > gpurun_out/e_skip2.log 2>&1 || { tail -30 gpurun_out/e_skip2.log; exit 1; }
for f in e_base e_skip1 e_skip2; do echo $f; grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/$f.log; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e -o run -- $B > gpurun_out/e_prof.log 2>&1 || { tail -30 gpurun_out/e_prof.log; exit 1; }
find gpurun_out/prof_e -name "*kernel_stats.csv" | head -3
