#!/bin/bash
# r03: training step, same-box A/B of write-through output stores: none / transfer-net Winograd convs
# (RST_TRAIN_WT=1) / those and the VGG convs (RST_LOSS_WT=1); the training / loss GPU tests with both on.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
RST_TRAIN_WT=1 RST_LOSS_WT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_loss.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ap.log 2>&1 || { tail -40 gpurun_out/pytest_ap.log; exit 1; }
tail -1 gpurun_out/pytest_ap.log
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 12"
for i in 1 2 3; do
  for w in 00 10 11; do
    RST_TRAIN_WT=${w:0:1} RST_LOSS_WT=${w:1:1} timeout -k 10 400 $T > gpurun_out/bench_ap_${w}_$i.log 2>&1 || { tail -30 gpurun_out/bench_ap_${w}_$i.log; exit 1; }
    echo "train_wt,loss_wt=$w run $i: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ap_${w}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
