#!/bin/bash
# Round-2 measurement pass: GPU tests, bench.py, rocprofv3 kernel stats of the inference frame loop and of
# the training step (B=4). Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 420 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -c 300 gpurun_out/bench.log
rm -rf gpurun_out/prof gpurun_out/prof_train
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 50 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor \
    --train-batch 0 > gpurun_out/bench_prof.log 2>&1 || { tail -30 gpurun_out/bench_prof.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- \
    python tools/train_step_run.py --steps 5 --transfer winograd_bf16x6 > gpurun_out/train_prof.log 2>&1 || { tail -30 gpurun_out/train_prof.log; exit 1; }
tail -3 gpurun_out/train_prof.log

rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- \
    python tools/wino_probe.py winograd_bf16x6 3 > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- \
    python tools/wino_probe.py winograd_bf16x6 3 > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
echo "pmc ok"
