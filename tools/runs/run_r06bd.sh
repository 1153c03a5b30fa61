#!/bin/bash
# r06bd: validation of the build with the env-gated race diagnostics (inactive by default) — GPU suite, smoke, two default
# bench lines, rocprof kernel trace of the headline + roofline recompute
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06bd bash tools/gpu_measure.sh tests smoke || exit 1
TAG=r06bd bash tools/gpu_measure.sh bench prof || exit 1
TAG=r06bd2 bash tools/gpu_measure.sh bench || exit 1
python tools/roofline_check.py $O/bench_r06bd.log $O/prof_r06bd/run_kernel_trace.csv > $O/roofline_check_r06bd.json; echo "roofline check rc=$?"
cat $O/roofline_check_r06bd.json
