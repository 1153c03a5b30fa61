#!/bin/bash
# r06n: how many CUs the start conv's weight gradient leaves to the predictor backward (RST_WGRAD9_FREE_CUS), the
# predictor backward's norm-output ring (RST_PBWD_DZR 3 vs one per unit), and a kernel + HIP API trace (host issue rate)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06n bash tools/gpu_measure.sh trainab=RST_WGRAD9_FREE_CUS=64@RST_WGRAD9_FREE_CUS=32@3 && \
TAG=r06o bash tools/gpu_measure.sh trainab=RST_WGRAD9_FREE_CUS=96@RST_WGRAD9_FREE_CUS=16@2 && \
TAG=r06p bash tools/gpu_measure.sh trainab=RST_WGRAD9_FREE_CUS=32:RST_PBWD_DZR=64@RST_WGRAD9_FREE_CUS=32@3 && \
RST_WGRAD9_FREE_CUS=32 TAG=r06n bash tools/gpu_measure.sh trainhip
