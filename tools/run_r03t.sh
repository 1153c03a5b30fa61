#!/bin/bash
# r03 checkpoint after the container re-creation: the whole GPU test suite, smoke(), the default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1 || { tail -40 gpurun_out/pytest_t.log; exit 1; }
tail -2 gpurun_out/pytest_t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_t.log 2>&1 || { tail -20 gpurun_out/smoke_t.log; exit 1; }
tail -2 gpurun_out/smoke_t.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_t.log 2>&1 || { tail -30 gpurun_out/bench_t.log; exit 1; }
tail -c 600 gpurun_out/bench_t.log
