#!/bin/bash
# r06as: what before the training leg slows it — full pre-training legs vs no PCIe leg vs short headline too (side legs
# after training are skipped in all three); then the expand_0 two-forms GPU test
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
C="--no-cpu-baseline --train-modes bf16 --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --no-two-styles"
for i in 1 2; do
  for v in a b c; do
    case $v in a) X="" ;; b) X="--pcie-steps 0" ;; c) X="--pcie-steps 0 --steps 5 --warmup 2" ;; esac
    timeout -k 10 400 python -u bench.py $C $X > $O/pre_r06as_${v}_$i.log 2>&1 || { tail -20 $O/pre_r06as_${v}_$i.log; exit 1; }
    echo "$v ($X) run $i: training $(grep -o '"training": {.\{0,420\}' $O/pre_r06as_${v}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_transfer.py -m gpu -v --timeout 300 --timeout-method thread \
    -k expand0_ksplit > $O/pytest_r06as.log 2>&1; echo "test rc=$?"; tail -2 $O/pytest_r06as.log
