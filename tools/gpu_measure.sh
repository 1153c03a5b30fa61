#!/bin/bash
# One GPU measurement pass (run on the GPU box via gpurun, from the repo root):
#   1. GPU parity tests (pytest -m gpu)            -> gpurun_out/pytest_gpu.log
#   2. bench.py (default flags)                      -> gpurun_out/bench.log
#   3. rocprofv3 --kernel-trace --stats of a short inference bench -> gpurun_out/prof/
#   4. two PMC passes (FETCH_SIZE, WRITE_SIZE) of tools/wino_probe.py -> gpurun_out/pmc_{f,w}/
# Every GPU step has its own time limit; the steps are chained so the first failure ends the call.
# Usage: bash tools/gpu_measure.sh [tests|bench|prof|pmc|all]...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(all)
want() { for s in "${steps[@]}"; do [ "$s" = "$1" ] || [ "$s" = all ] && return 0; done; return 1; }

if want tests; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
    tail -3 gpurun_out/pytest_gpu.log
fi
if want bench; then
    timeout -k 10 420 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
    tail -c 600 gpurun_out/bench.log
fi
if want prof; then
    rm -rf gpurun_out/prof
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python bench.py --steps 50 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor \
        --train-batch 0 --no-two-styles > gpurun_out/bench_prof.log 2>&1 || { tail -30 gpurun_out/bench_prof.log; exit 1; }
    echo "prof ok"
fi
if want pmc; then
    rm -rf gpurun_out/pmc_f gpurun_out/pmc_w
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- \
        python tools/wino_probe.py winograd_bf16x6 3 > gpurun_out/pmc_f.log 2>&1 || { tail -20 gpurun_out/pmc_f.log; exit 1; }
    timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- \
        python tools/wino_probe.py winograd_bf16x6 3 > gpurun_out/pmc_w.log 2>&1 || { tail -20 gpurun_out/pmc_w.log; exit 1; }
    echo "pmc ok"
fi
