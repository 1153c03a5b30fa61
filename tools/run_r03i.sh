#!/bin/bash
# r03 checkpoint: the whole GPU test suite, smoke(), and the default bench line (as the driver runs it).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1 || { tail -40 gpurun_out/pytest_i.log; exit 1; }
tail -2 gpurun_out/pytest_i.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_i.log 2>&1 || { tail -20 gpurun_out/smoke_i.log; exit 1; }
tail -2 gpurun_out/smoke_i.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_i.log 2>&1 || { tail -30 gpurun_out/bench_i.log; exit 1; }
tail -c 600 gpurun_out/bench_i.log
timeout -k 10 120 tools/conv_bench 4 vgg > gpurun_out/conv_bench_vgg_i.log 2>&1 || { tail -20 gpurun_out/conv_bench_vgg_i.log; exit 1; }
cat gpurun_out/conv_bench_vgg_i.log
