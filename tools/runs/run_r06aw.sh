#!/bin/bash
# r06aw: final validation of the committed build (fin_sigmoid3 load order included) — GPU suite, smoke, two default
# bench lines, rocprof kernel trace of the headline + roofline recompute
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06aw bash tools/gpu_measure.sh tests smoke || exit 1
TAG=r06aw bash tools/gpu_measure.sh bench prof || exit 1
TAG=r06aw2 bash tools/gpu_measure.sh bench || exit 1
python tools/roofline_check.py $O/bench_r06aw.log $O/prof_r06aw/run_kernel_trace.csv > $O/roofline_check_r06aw.json; echo "roofline check rc=$?"
cat $O/roofline_check_r06aw.json
