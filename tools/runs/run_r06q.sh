#!/bin/bash
# r06q: loss targets issued after the predictor forward (RST_TARGETS_AFTER_PFWD) and the start-conv weight gradient's
# free CUs beyond 96; the full-size captured step vs eager (tools/train_graph_check.py)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
export RST_WGRAD9_FREE_CUS=96
TAG=r06q bash tools/gpu_measure.sh trainab=RST_TARGETS_AFTER_PFWD=1@-@3 && \
TAG=r06r bash tools/gpu_measure.sh trainab=RST_WGRAD9_FREE_CUS=128@RST_WGRAD9_FREE_CUS=160@2 && \
timeout -k 10 300 python -u tools/train_graph_check.py 4 10 > gpurun_out/graph_r06q.log 2>&1 && tail -2 gpurun_out/graph_r06q.log && \
TAG=r06q bash tools/gpu_measure.sh trainprof
