#!/bin/bash
# r03 end-of-round measurement of HEAD (write-through output stores on): PMC traffic passes -> traffic json,
# full GPU suite, smoke, default bench line (with the fresh traffic), rocprofv3 kernel stats of the frame loop.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_measure.sh pmc || exit 1
F=$(find gpurun_out/pmc_f -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/pmc_w -name '*counter_collection.csv' | head -1)
python tools/pmc_traffic.py "$F" "$W" gpurun_out/traffic_r03.json || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_final3.log 2>&1 || { tail -40 gpurun_out/pytest_final3.log; exit 1; }
tail -1 gpurun_out/pytest_final3.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final3.log 2>&1 || { tail -30 gpurun_out/smoke_final3.log; exit 1; }
tail -2 gpurun_out/smoke_final3.log
timeout -k 10 900 python -u bench.py --traffic-json gpurun_out/traffic_r03.json > gpurun_out/bench_final3.log 2>&1 || { tail -30 gpurun_out/bench_final3.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "frames/s"' gpurun_out/bench_final3.log | head -1
bash tools/gpu_measure.sh prof || exit 1
