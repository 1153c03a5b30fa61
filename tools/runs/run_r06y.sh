#!/bin/bash
# r06y: 16x16-pixel x 128 VGG16 conv tiles (RST_BF3_BIG = minimum workgroup count; 324 registers, one workgroup per
# CU) against the 8x16 tiles: loss tests with the big tiles forced on, then training-step A/B
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
RST_BF3_BIG=1 TAG=r06y bash tools/gpu_measure.sh "tests=loss or bf16" && \
TAG=r06y bash tools/gpu_measure.sh trainab=RST_BF3_BIG=400@-@3
