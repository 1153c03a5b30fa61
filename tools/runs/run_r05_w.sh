#!/bin/bash
# round 5: SQ passes of the frame (start conv F(3x3) included) and HBM FETCH/WRITE passes of the frame probe on the
# final residual-conv build; the training step's kernel trace (bench training leg only)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05w bash tools/gpu_measure.sh sq=frame pmc || exit 1
rm -rf gpurun_out/trainprof_r05w
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trainprof_r05w -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest \
  --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 10 > gpurun_out/trainprof_r05w.log 2>&1 || { tail -30 gpurun_out/trainprof_r05w.log; exit 1; }
grep -o '"training": {.\{0,300\}' gpurun_out/trainprof_r05w.log | head -2
