#!/bin/bash
# r06ac: the loss targets' VGG16 layers as one-image launches (RST_TARGETS_PER_IMAGE=1): loss tests with it on,
# training-step A/B, step phases (the predictor's forward beside the targets)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
RST_TARGETS_PER_IMAGE=1 TAG=r06ac bash tools/gpu_measure.sh "tests=loss or train_step_matches or joint" && \
TAG=r06ac bash tools/gpu_measure.sh trainab=RST_TARGETS_PER_IMAGE=1@-@3 && \
RST_TARGETS_PER_IMAGE=1 timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06ac_pi.log 2>&1 && cat gpurun_out/phases_r06ac_pi.log
