#!/bin/bash
# r03 pass: inference with every CIN's statistics through f64 accumulators (parallel slot merge in the
# consumers, zeroed by the start conv): inference GPU tests, the inference bench and its kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_transfer.py tests/test_gpu_configs.py tests/test_gpu_entry_scripts.py \
    tests/test_gpu_predictor.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_g.log 2>&1 || { tail -40 gpurun_out/pytest_g.log; exit 1; }
tail -2 gpurun_out/pytest_g.log
B="python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --stream-batch 8 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --train-batch 0"
timeout -k 10 300 $B > gpurun_out/bench_g.log 2>&1 || { tail -30 gpurun_out/bench_g.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/bench_g.log
grep -o '"two_styles": {.\{0,300\}' gpurun_out/bench_g.log
grep -o '"stream": {.\{0,300\}' gpurun_out/bench_g.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g -o run -- $B --stream-batch 0 --no-two-styles > gpurun_out/prof_g.log 2>&1 || { tail -30 gpurun_out/prof_g.log; exit 1; }
ls gpurun_out/prof_g
