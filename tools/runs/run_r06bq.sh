#!/bin/bash
# r06bq: the final tree's GPU suite (with the two-stream co-residency test) and smoke
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06bq bash tools/gpu_measure.sh tests smoke
