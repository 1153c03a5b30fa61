#!/bin/bash
# r03 pass: bank-conflict-free strides for the 9x9 weight-gradient kernels (wgrad9 / wgradT9): training GPU
# tests, the config-4 training bench line and its kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1 || { tail -40 gpurun_out/pytest_l.log; exit 1; }
tail -2 gpurun_out/pytest_l.log
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10"
timeout -k 10 300 $B > gpurun_out/bench_l.log 2>&1 || { tail -30 gpurun_out/bench_l.log; exit 1; }
grep -o '"training": {.\{0,420\}' gpurun_out/bench_l.log | grep -o '"ms_per_step": [0-9.]*'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_l -o run -- $B > gpurun_out/prof_l.log 2>&1 || { tail -30 gpurun_out/prof_l.log; exit 1; }
ls gpurun_out/prof_l
