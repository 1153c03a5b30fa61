#!/bin/bash
# r06bm: validation of the final build (scalar-FMA last conv for training) — GPU suite, smoke, two default
# bench lines, rocprof kernel trace of the headline + roofline recompute
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06bm bash tools/gpu_measure.sh tests smoke || exit 1
TAG=r06bm bash tools/gpu_measure.sh bench prof || exit 1
TAG=r06bm2 bash tools/gpu_measure.sh bench || exit 1
python tools/roofline_check.py $O/bench_r06bm.log $O/prof_r06bm/run_kernel_trace.csv > $O/roofline_check_r06bm.json; echo "roofline check rc=$?"
cat $O/roofline_check_r06bm.json
