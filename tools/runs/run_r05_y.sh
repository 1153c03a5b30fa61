#!/bin/bash
# round 5: kernel trace of the training step with conv_vgg.hip (does it run, and how long per layer)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/trainprof_r05y
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trainprof_r05y -o run -- \
  python bench.py --steps 2 --warmup 1 --settle-s 0 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest \
  --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 4 > gpurun_out/trainprof_r05y.log 2>&1 || { tail -30 gpurun_out/trainprof_r05y.log; exit 1; }
grep -o '"training": {.\{0,400\}' gpurun_out/trainprof_r05y.log | grep -o 'ms_per_step": [0-9.]*'
