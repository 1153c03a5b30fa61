#!/bin/bash
# r06aj: the BN merge reverted — the training file in order (the 480x960 bf16-VGG parity test failed after the joint
# predictor tests with the merge on), the whole GPU suite, smoke, the default bench line
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
PYTEST_X=" " TAG=r06aj1 bash tools/gpu_measure.sh "tests=test_gpu_train" || exit 1
TAG=r06aj bash tools/gpu_measure.sh tests smoke bench
