#!/bin/bash
# r06aq: validation of the round's build after the second session — GPU suite, smoke, FETCH / WRITE passes -> traffic of
# this build, the default bench line with that traffic, rocprof kernel trace of the headline + the roofline recompute,
# training kernel stats
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06aq bash tools/gpu_measure.sh tests smoke pmc || exit 1
python tools/pmc_traffic.py $O/pmc_f_r06aq/run_counter_collection.csv $O/pmc_w_r06aq/run_counter_collection.csv \
    $O/traffic_r06aq.json > $O/traffic_r06aq.log 2>&1 || { tail -20 $O/traffic_r06aq.log; exit 1; }
TAG=r06aq bash tools/gpu_measure.sh bench=--traffic-json,$O/traffic_r06aq.json prof || exit 1
python tools/roofline_check.py $O/bench_r06aq.log $O/prof_r06aq/run_kernel_trace.csv > $O/roofline_check_r06aq.json; echo "roofline check rc=$?"
cat $O/roofline_check_r06aq.json
TAG=r06aq bash tools/gpu_measure.sh trainprof
# the predictor's BN finalize loops unrolled (loads of 8 / 4 partials in flight) against the rolled loops (var_ptold)
TAG=r06aq bash tools/gpu_measure.sh trainab=RST_LIB=tools/var_ptold.so@-@3
