#!/bin/bash
# r06i: the loss targets' stream leaving CUs to the predictor forward (RST_TARGETS_FREE_CUS 32 / 64) vs unmasked
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06i bash tools/gpu_measure.sh trainab=RST_TARGETS_FREE_CUS=32@-@3 &&
TAG=r06j bash tools/gpu_measure.sh trainab=RST_TARGETS_FREE_CUS=64@RST_TARGETS_FREE_CUS=16@3
