#!/bin/bash
# r06c: GPU suite, short bench (in-graph roofline) + rocprof trace, fused start-conv tail A/B, bf16 VGG activation
# training A/B; last (a crash ends the call): which stream overlap breaks the whole-step graph capture
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
TAG=r06c bash tools/gpu_measure.sh tests short prof ab=RST_F3_FUSED_TAIL=0@-@3 trainab=RST_VGG_ACT_F32=1@-@3 || exit 1
S="RST_SERIAL_TARGETS=1 RST_SERIAL_PREDICTOR_BWD=1 RST_SERIAL_PREDICTOR_WGRAD=1"
env $S timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06c_serial.log 2>&1; echo "serial rc=$?"; tail -2 $O/graph_r06c_serial.log
env RST_SERIAL_PREDICTOR_BWD=1 RST_SERIAL_PREDICTOR_WGRAD=1 timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06c_targets.log 2>&1 &&
env RST_SERIAL_PREDICTOR_WGRAD=1 timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06c_pbwd.log 2>&1 &&
timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06c_default.log 2>&1
echo "graph checks rc=$?"; tail -2 $O/graph_r06c_*.log
