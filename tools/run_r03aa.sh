#!/bin/bash
# r03: VGG16 128-wide conv tiles on config 136 (two-stage weight prefetch): loss/train GPU tests, training line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_aa.log 2>&1 || { tail -40 gpurun_out/pytest_aa.log; exit 1; }
tail -1 gpurun_out/pytest_aa.log
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10"
for i in 1 2; do
  timeout -k 10 400 $T > gpurun_out/bench_aa_$i.log 2>&1 || { tail -30 gpurun_out/bench_aa_$i.log; exit 1; }
  echo "training: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_aa_$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_aa -o run -- $T > gpurun_out/prof_aa.log 2>&1 || { tail -30 gpurun_out/prof_aa.log; exit 1; }
echo done
