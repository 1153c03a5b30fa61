#!/bin/bash
# r06av: last_x6's fill with all three row loads in flight before the first store — the micro-bench (old / new, with the
# LAST_PROF timeline), kernel time in the frame (rocprof), headline pairs against the previous build
# (tools/var_lastold.so), and the transfer GPU tests
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in old new old new; do timeout -k 10 60 tools/last_r06av_$v 200 >> gpurun_out/lastbench_r06av_$v.log 2>&1 || exit 1; done && \
TAG=r06av bash tools/gpu_measure.sh prof && \
TAG=r06av bash tools/gpu_measure.sh ab=RST_LIB=tools/var_lastold.so@-@3 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "transfer or configs or last" \
    > gpurun_out/pytest_r06av.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/pytest_r06av.log
