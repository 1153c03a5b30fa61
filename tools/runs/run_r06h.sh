#!/bin/bash
# r06h: bf16-gradient staging tiles (146 / 147) and the predictor backward's batched weight transpose: loss / training /
# predictor GPU tests, A/B of the bf16 gradients, training trace
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06h bash tools/gpu_measure.sh "tests=loss or train or predictor" trainab=RST_VGG_GRAD_F32=1@-@3 trainprof
