#!/bin/bash
# r06ae: the in-graph timeline test
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06ae bash tools/gpu_measure.sh "tests=timeline or l2_weight"
