#!/bin/bash
# r03 pass: (1) training with the x6 start conv (wino9_x6 training mode), (2) inference with the residual
# convs' CIN statistics through f64 accumulators (no finalize kernels between them): GPU tests, the short
# bench (inference + config-4 training line) and its kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transfer.py tests/test_gpu_configs.py -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_f1.log 2>&1 || { tail -40 gpurun_out/pytest_f1.log; exit 1; }
tail -2 gpurun_out/pytest_f1.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_distributed.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_f2.log 2>&1 || { tail -40 gpurun_out/pytest_f2.log; exit 1; }
tail -2 gpurun_out/pytest_f2.log
B="python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --train-modes bf16 --train-steps 10"
timeout -k 10 300 $B > gpurun_out/bench_f.log 2>&1 || { tail -30 gpurun_out/bench_f.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/bench_f.log
grep -o '"two_styles": {.\{0,300\}' gpurun_out/bench_f.log
grep -o '"training": {.\{0,400\}' gpurun_out/bench_f.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f -o run -- $B > gpurun_out/prof_f.log 2>&1 || { tail -30 gpurun_out/prof_f.log; exit 1; }
ls gpurun_out/prof_f
