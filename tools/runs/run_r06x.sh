#!/bin/bash
# r06x: the bf16 Gram staging with conflict-free stores and a one-chunk load prefetch: loss / Gram / training GPU tests,
# SQ passes of the training step (Gram duration and lds_conflict against r06w), training step
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06x bash tools/gpu_measure.sh "tests=loss or gram or train" sq=train trainab=-@-@2
