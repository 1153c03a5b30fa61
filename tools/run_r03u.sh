#!/bin/bash
# r03: wino_x6w (16x16 px x 64 channels per workgroup) against wino_x6 and f32 wino standalone, the transfer GPU
# tests on the library (wino_x6w in inference), then a short bench line with and without RST_X6_NARROW.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "1 128 1" "1 128 3" "1 128 2" "1 32 0" "1 128 1 1" "1 128 3 1" "2 128 3 0 65 97"; do
  echo "== wino_x6w_bench $args"
  timeout -k 10 60 tools/wino_x6w_bench $args || { echo "FAILED rc=$?"; exit 1; }
done > gpurun_out/x6w_u.log 2>&1 || { cat gpurun_out/x6w_u.log; exit 1; }
cat gpurun_out/x6w_u.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_transfer.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1 || { tail -40 gpurun_out/pytest_u.log; exit 1; }
tail -2 gpurun_out/pytest_u.log
B="python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --train-batch 0"
timeout -k 10 300 $B > gpurun_out/bench_u_wide.log 2>&1 || { tail -30 gpurun_out/bench_u_wide.log; exit 1; }
RST_X6_NARROW=1 timeout -k 10 300 $B > gpurun_out/bench_u_narrow.log 2>&1 || { tail -30 gpurun_out/bench_u_narrow.log; exit 1; }
timeout -k 10 300 $B > gpurun_out/bench_u_wide2.log 2>&1 || { tail -30 gpurun_out/bench_u_wide2.log; exit 1; }
for f in wide narrow wide2; do grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/bench_u_$f.log; grep -o '"two_styles": {.\{0,120\}' gpurun_out/bench_u_$f.log | head -1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_u -o run -- $B > gpurun_out/prof_u.log 2>&1 || { tail -30 gpurun_out/prof_u.log; exit 1; }
ls gpurun_out/prof_u
