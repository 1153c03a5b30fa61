#!/bin/bash
# r03 pass: transfer/predictor/entry-script GPU tests (fused output kernel, two-style blends), the short frame
# bench, and the residual kernel's s_setprio variants (standalone bench). Each GPU step has its own limit.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_transfer.py tests/test_gpu_entry_scripts.py tests/test_gpu_configs.py \
    tests/test_gpu_predictor.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_d.log 2>&1 || { tail -30 gpurun_out/pytest_d.log; exit 1; }
tail -2 gpurun_out/pytest_d.log
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 \
    --no-predictor --train-batch 0 --no-ingest --pcie-steps 0 > gpurun_out/bench_d.log 2>&1 || { tail -30 gpurun_out/bench_d.log; exit 1; }
tail -c 300 gpurun_out/bench_d.log; echo
rm -f gpurun_out/x6p.log
for b in wino_x6_bench_v3 wino_x6_bench_p1 wino_x6_bench_p2 wino_x6_bench_v3; do
    for args in "1 128 1 0 0 0 0 1" "1 128 3" "1 128 3 3 0 0 1"; do
        echo "== $b $args" >> gpurun_out/x6p.log
        timeout -k 5 60 tools/$b $args >> gpurun_out/x6p.log 2>&1 || { tail -20 gpurun_out/x6p.log; exit 1; }
    done
done
grep "==\|wino_x6 B" gpurun_out/x6p.log
