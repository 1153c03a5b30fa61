#!/bin/bash
# r03: wino_x6 write-through (sc1) output / materialised-input stores, same-box A/B (RST_WT_STORES bits: 1 wino_x6 output, 2 its materialised input, 4 wino9_x6 output, 8 conv_lite output) of the
# B=1 frame and the B=8 stream graph; the GPU suite under the default (13).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_an.log 2>&1 || { tail -40 gpurun_out/pytest_an.log; exit 1; }
tail -1 gpurun_out/pytest_an.log
T="python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-batch 0"
for i in 1 2 3 4; do
  for w in 0 13; do
    RST_WT_STORES=$w timeout -k 10 400 $T > gpurun_out/bench_an_${w}_$i.log 2>&1 || { tail -30 gpurun_out/bench_an_${w}_$i.log; exit 1; }
    echo "wt=$w run $i: $(grep -o '"value": [0-9.]*' gpurun_out/bench_an_${w}_$i.log | head -1) stream $(grep -o '"stream_graph": {"fps": [0-9.]*' gpurun_out/bench_an_${w}_$i.log)"
  done
done
