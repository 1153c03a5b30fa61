#!/bin/bash
# r03: loss targets on the trainer's side stream (beside the predictor / transfer forward): training GPU tests,
# training line with and without (RST_SERIAL_TARGETS=1), kernel trace of the training leg.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_predictor_train.py tests/test_gpu_distributed.py tests/test_gpu_entry_scripts.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_y.log 2>&1 || { tail -40 gpurun_out/pytest_y.log; exit 1; }
tail -1 gpurun_out/pytest_y.log
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10"
for i in 1 2; do
  timeout -k 10 400 $T > gpurun_out/bench_y_on$i.log 2>&1 || { tail -30 gpurun_out/bench_y_on$i.log; exit 1; }
  RST_SERIAL_TARGETS=1 timeout -k 10 400 $T > gpurun_out/bench_y_off$i.log 2>&1 || { tail -30 gpurun_out/bench_y_off$i.log; exit 1; }
  echo "overlap: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_y_on$i.log | grep -o '"ms_per_step": [0-9.]*')   serial: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_y_off$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
