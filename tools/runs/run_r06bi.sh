#!/bin/bash
# r06bi: validation of the last build (env-gated dump / exclusive-CU diagnostics added) — GPU suite, smoke, default bench
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06bi bash tools/gpu_measure.sh tests smoke bench
