#!/bin/bash
# r06d: training step kernel traces with f32 / bf16 VGG16 activation storage (bf16 staging tiles 144 / 145), their A/B,
# PMC traffic passes of the frame; last: the whole-step graph capture with every overlap on (fresh fork/join events)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
RST_VGG_ACT_F32=1 TAG=r06d_f32 bash tools/gpu_measure.sh trainprof &&
TAG=r06d_bf16 bash tools/gpu_measure.sh trainprof &&
TAG=r06d bash tools/gpu_measure.sh trainab=RST_VGG_ACT_F32=1@-@3 pmc &&
timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06d_default.log 2>&1
echo "graph check rc=$?"; tail -n 2 $O/graph_r06d_default.log
