#!/bin/bash
# r03 end-of-round check of HEAD (training write-through defaults): full GPU suite, smoke, default bench line.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final4.log 2>&1 || { tail -40 gpurun_out/pytest_final4.log; exit 1; }
tail -1 gpurun_out/pytest_final4.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final4.log 2>&1 || { tail -30 gpurun_out/smoke_final4.log; exit 1; }
tail -2 gpurun_out/smoke_final4.log
timeout -k 10 900 python -u bench.py  > gpurun_out/bench_final4.log 2>&1 || { tail -30 gpurun_out/bench_final4.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s"' gpurun_out/bench_final4.log | head -1
