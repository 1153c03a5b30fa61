#!/bin/bash
# r03 final: whole GPU suite, smoke(), the driver's bench invocation (--steps 20 --warmup 5) and the default one.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { tail -40 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -2 gpurun_out/smoke_final.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_driverlike.log 2>&1 || { tail -30 gpurun_out/bench_driverlike.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/bench_driverlike.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default_final.log 2>&1 || { tail -30 gpurun_out/bench_default_final.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s", "n_gpus"' gpurun_out/bench_default_final.log
