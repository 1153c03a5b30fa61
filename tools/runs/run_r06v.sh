#!/bin/bash
# r06v: validation of the round's final build — GPU suite, smoke, FETCH / WRITE passes -> traffic of this build, the
# default bench line (with that traffic), rocprof kernel trace of the headline + the roofline recompute, training stats
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06v bash tools/gpu_measure.sh tests smoke pmc || exit 1
python tools/pmc_traffic.py $O/pmc_f_r06v/run_counter_collection.csv $O/pmc_w_r06v/run_counter_collection.csv \
    $O/traffic_r06v.json > $O/traffic_r06v.log 2>&1 || { tail -20 $O/traffic_r06v.log; exit 1; }
TAG=r06v bash tools/gpu_measure.sh bench=--traffic-json,$O/traffic_r06v.json prof || exit 1
python tools/roofline_check.py $O/bench_r06v.log $O/prof_r06v/run_kernel_trace.csv > $O/roofline_check_r06v.json; echo "roofline check rc=$?"
cat $O/roofline_check_r06v.json
TAG=r06v bash tools/gpu_measure.sh trainprof
