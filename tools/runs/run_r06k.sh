#!/bin/bash
# r06k: the start conv's weight gradient (one 102 KB-LDS workgroup per CU) left no CU to the predictor backward for its
# 1.1 ms (profiles/r06/r06h trace): A/B of leaving 32 CUs free, of the predictor backward's streams at high priority, and
# of both; training trace with both
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06k bash tools/gpu_measure.sh trainab=RST_WGRAD9_FREE_CUS=32@-@3 && \
TAG=r06l bash tools/gpu_measure.sh trainab=RST_PBWD_PRIORITY=1@-@3 && \
TAG=r06m bash tools/gpu_measure.sh trainab=RST_WGRAD9_FREE_CUS=32:RST_PBWD_PRIORITY=1@RST_WGRAD9_FREE_CUS=64:RST_PBWD_PRIORITY=1@3 && \
RST_WGRAD9_FREE_CUS=32 RST_PBWD_PRIORITY=1 TAG=r06k bash tools/gpu_measure.sh trainprof
