#!/bin/bash
# r03: training forward with the next residual conv's U touched into L2 (A/B: RST_NO_U_PREFETCH=1), train tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ak.log 2>&1 || { tail -40 gpurun_out/pytest_ak.log; exit 1; }
tail -1 gpurun_out/pytest_ak.log
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 12"
for i in 1 2 3; do
  timeout -k 10 400 $T > gpurun_out/bench_ak_on$i.log 2>&1 || { tail -30 gpurun_out/bench_ak_on$i.log; exit 1; }
  RST_NO_U_PREFETCH=1 timeout -k 10 400 $T > gpurun_out/bench_ak_off$i.log 2>&1 || { tail -30 gpurun_out/bench_ak_off$i.log; exit 1; }
  echo "touch: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ak_on$i.log | grep -o '"ms_per_step": [0-9.]*')   none: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ak_off$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
