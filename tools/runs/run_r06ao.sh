#!/bin/bash
# r06ao: config-4 step pairs for the tap-row residual weight gradient (RST_WGRAD_X6R=0: the 128-row x6 kernel), then the
# current build's GPU suite, smoke and default bench line
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06ao bash tools/gpu_measure.sh trainab=RST_WGRAD_X6R=0@-@3 && \
TAG=r06ao bash tools/gpu_measure.sh tests smoke bench
