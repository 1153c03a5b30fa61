#!/bin/bash
# r06ah: the predictor's BatchNorm finalizes merged into the last workgroup of their stats / reduce launches
# (68 fewer dispatches per training step) — predictor / training GPU tests, then config-4 step A/B pairs
# (RST_BN_MERGE=0 restores the finalize launches)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06ah bash tools/gpu_measure.sh "tests=predictor or train" || exit 1
TAG=r06ah bash tools/gpu_measure.sh trainab=RST_BN_MERGE=0@-@3
