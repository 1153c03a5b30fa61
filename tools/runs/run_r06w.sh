#!/bin/bash
# r06w: SQ counter passes of the training step (MFMA busy, stalls, LDS) for the VGG16 conv tiles
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06w bash tools/gpu_measure.sh sq=train
