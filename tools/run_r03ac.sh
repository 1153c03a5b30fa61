#!/bin/bash
# r03: predictor-training BN finalize per channel quad: predictor/train GPU tests, training line, training trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_predictor_train.py tests/test_gpu_train.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ac.log 2>&1 || { tail -40 gpurun_out/pytest_ac.log; exit 1; }
tail -1 gpurun_out/pytest_ac.log
T="python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10"
for i in 1 2; do
  timeout -k 10 400 $T > gpurun_out/bench_ac_$i.log 2>&1 || { tail -30 gpurun_out/bench_ac_$i.log; exit 1; }
  echo "training: $(grep -o '"training": {.\{0,420\}' gpurun_out/bench_ac_$i.log | grep -o '"ms_per_step": [0-9.]*')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ac -o run -- $T > gpurun_out/prof_ac.log 2>&1 || { tail -30 gpurun_out/prof_ac.log; exit 1; }
echo done
