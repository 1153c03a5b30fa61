#!/bin/bash
# r06au: the final CIN + sigmoid kernel with its data loads issued before the affine merge — kernel time in the frame
# (rocprof) and headline pairs against the previous form (tools/var_normold.so)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06au bash tools/gpu_measure.sh prof && \
TAG=r06au bash tools/gpu_measure.sh ab=RST_LIB=tools/var_normold.so@-@3 && \
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "transfer or configs" \
    > gpurun_out/pytest_r06au.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/pytest_r06au.log
