#!/bin/bash
# r03: next-layer weights into L2 for every inference layer kind (wino9_x6, conv_lite, wino_x6): transfer GPU tests,
# headline runs with and without (RST_NO_U_PREFETCH=1), kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_transfer.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_x.log 2>&1 || { tail -40 gpurun_out/pytest_x.log; exit 1; }
tail -1 gpurun_out/pytest_x.log
B="python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --train-batch 0 --no-two-styles"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/bench_x_on$i.log 2>&1 || { tail -30 gpurun_out/bench_x_on$i.log; exit 1; }
  RST_NO_U_PREFETCH=1 timeout -k 10 300 $B > gpurun_out/bench_x_off$i.log 2>&1 || { tail -30 gpurun_out/bench_x_off$i.log; exit 1; }
  echo "on:  $(grep -o '"value": [0-9.]*, "unit": "frames/s"' gpurun_out/bench_x_on$i.log)   off: $(grep -o '"value": [0-9.]*, "unit": "frames/s"' gpurun_out/bench_x_off$i.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x_on -o run -- $B > gpurun_out/prof_x_on.log 2>&1 || { tail -30 gpurun_out/prof_x_on.log; exit 1; }
echo done
