#!/bin/bash
# r06at: final validation of the round's build — GPU suite (incl. the expand_0 two-forms test), smoke, the default
# bench line (training leg now before the side legs), rocprof kernel trace of the headline + roofline recompute
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06at bash tools/gpu_measure.sh tests smoke || exit 1
TAG=r06at bash tools/gpu_measure.sh bench prof || exit 1
python tools/roofline_check.py $O/bench_r06at.log $O/prof_r06at/run_kernel_trace.csv > $O/roofline_check_r06at.json; echo "roofline check rc=$?"
cat $O/roofline_check_r06at.json
