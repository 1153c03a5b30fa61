#!/bin/bash
# r06g: bf16 VGG16 gradients (mixed_bfloat16): loss / training GPU tests, A/B against f32 gradients, training trace
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06g bash tools/gpu_measure.sh "tests=loss or train" trainab=RST_VGG_GRAD_F32=1@-@3 trainprof
