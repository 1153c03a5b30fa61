#!/bin/bash
# r06z: the config-4 bf16 VGG16 line against its float32 simulation at the bench's full 480x960 (+ loss tests), then
# the loss targets' VGG16 convs requesting more LDS per workgroup (RST_TARGETS_LDS) so that fewer are resident per CU
# beside the style predictor's forward: 1 per CU (81920 B) and 2 per CU (54000 B) against none; step phases
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
PYTEST_X=" " TAG=r06z bash tools/gpu_measure.sh "tests=at_scale or loss"
head -c 1500 gpurun_out/train_parity_scale_full_bf16_winograd_bf16x6.json; echo
TAG=r06aa bash tools/gpu_measure.sh trainab=RST_TARGETS_LDS=81920@-@3 && \
TAG=r06ab bash tools/gpu_measure.sh trainab=RST_TARGETS_LDS=54000@-@2 && \
RST_TARGETS_LDS=81920 timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06aa_lds.log 2>&1 && cat gpurun_out/phases_r06aa_lds.log && \
timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06aa_default.log 2>&1 && cat gpurun_out/phases_r06aa_default.log
