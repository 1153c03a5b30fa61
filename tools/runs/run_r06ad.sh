#!/bin/bash
# r06ad: one-image launches for the style target's VGG16 pass only (RST_TARGETS_PER_IMAGE=2) and for both (=1)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06ad bash tools/gpu_measure.sh trainab=RST_TARGETS_PER_IMAGE=2@-@3 && \
RST_TARGETS_PER_IMAGE=2 timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06ad_pi2.log 2>&1 && cat gpurun_out/phases_r06ad_pi2.log && \
timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06ad_default.log 2>&1 && cat gpurun_out/phases_r06ad_default.log
