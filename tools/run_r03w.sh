#!/bin/bash
# r03: next-layer U prefetch in the residual convs (A/B: RST_NO_U_PREFETCH=1) and the VGG16 max pool fused into the
# conv_bf3 epilogue — transfer/loss/train GPU tests, alternating headline runs, training line, kernel traces.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_transfer.py tests/test_gpu_loss.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_w.log 2>&1 || { tail -40 gpurun_out/pytest_w.log; exit 1; }
tail -1 gpurun_out/pytest_w.log
B="python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --train-batch 0 --no-two-styles"
for i in 1 2 3; do
  timeout -k 10 300 $B > gpurun_out/bench_w_on$i.log 2>&1 || { tail -30 gpurun_out/bench_w_on$i.log; exit 1; }
  RST_NO_U_PREFETCH=1 timeout -k 10 300 $B > gpurun_out/bench_w_off$i.log 2>&1 || { tail -30 gpurun_out/bench_w_off$i.log; exit 1; }
  echo "on:  $(grep -o '"value": [0-9.]*, "unit": "frames/s"' gpurun_out/bench_w_on$i.log)   off: $(grep -o '"value": [0-9.]*, "unit": "frames/s"' gpurun_out/bench_w_off$i.log)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w_on -o run -- $B > gpurun_out/prof_w_on.log 2>&1 || { tail -30 gpurun_out/prof_w_on.log; exit 1; }
RST_NO_U_PREFETCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w_off -o run -- $B > gpurun_out/prof_w_off.log 2>&1 || { tail -30 gpurun_out/prof_w_off.log; exit 1; }
T="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10"
timeout -k 10 400 $T > gpurun_out/bench_w_train.log 2>&1 || { tail -30 gpurun_out/bench_w_train.log; exit 1; }
grep -o '"training": {.\{0,420\}' gpurun_out/bench_w_train.log | grep -o '"ms_per_step": [0-9.]*'
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w_train -o run -- $T > gpurun_out/prof_w_train.log 2>&1 || { tail -30 gpurun_out/prof_w_train.log; exit 1; }
find gpurun_out/prof_w_on gpurun_out/prof_w_off gpurun_out/prof_w_train -name "*kernel_stats.csv"
