#!/bin/bash
# r03: training step, same-box A/B of write-through stores: RST_TRAIN_WT 1 (Winograd conv outputs, the default)
# / 5 (+ the other transfer convs) / 9 (+ the VGG16 input gradients) / 13 (both); the training GPU tests under 15.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
RST_TRAIN_WT=15 timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ar.log 2>&1 || { tail -40 gpurun_out/pytest_ar.log; exit 1; }
tail -1 gpurun_out/pytest_ar.log
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 12"
for i in 1 2 3; do
  for w in 1 5 9 13; do
    RST_TRAIN_WT=$w timeout -k 10 400 $T > gpurun_out/bench_ar_${w}_$i.log 2>&1 || { tail -30 gpurun_out/bench_ar_${w}_$i.log; exit 1; }
    echo "train_wt=$w run $i: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ar_${w}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
