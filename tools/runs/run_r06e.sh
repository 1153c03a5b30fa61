#!/bin/bash
# r06e: Gram on bf16 features with 8-B staging loads; loss / training GPU tests, training A/B and trace; last: graph
# capture with the predictor's weight-gradient overlap but a serial predictor backward (is the nested join the crash?)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06e bash tools/gpu_measure.sh "tests=loss or train" trainab=RST_VGG_ACT_F32=1@-@3 trainprof &&
env RST_SERIAL_PREDICTOR_BWD=1 timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06e_wgrad_only.log 2>&1
echo "graph check rc=$?"; tail -n 2 $O/graph_r06e_wgrad_only.log
