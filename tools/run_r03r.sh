#!/bin/bash
# r03 pass: block1_conv1 on bf16 operands (plain-bf16 loss): loss + training GPU tests, short bench, training trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out

timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_train.py \
    -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r.log 2>&1 || { tail -40 gpurun_out/pytest_r.log; exit 1; }
tail -2 gpurun_out/pytest_r.log
B="python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10"
timeout -k 10 300 $B > gpurun_out/bench_r.log 2>&1 || { tail -30 gpurun_out/bench_r.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/bench_r.log
grep -o '"training": {.\{0,420\}' gpurun_out/bench_r.log | grep -o '"ms_per_step": [0-9.]*'
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r -o run -- $B > gpurun_out/prof_r.log 2>&1 || { tail -30 gpurun_out/prof_r.log; exit 1; }
ls gpurun_out/prof_r
