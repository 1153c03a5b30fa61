#!/bin/bash
# r06f: instruction-cache experiment on the residual conv (warm vs cycling templates, in-graph shares); the whole-step
# graph-capture GPU test (predictor backward serial under capture); training step trace of this build
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 ./tools/icache_x6 50 > $O/icache_r06f.log 2>&1 && cat $O/icache_r06f.log &&
TAG=r06f bash tools/gpu_measure.sh "tests=graph_replay or bitwise" &&
timeout -k 10 120 python -u tools/train_graph_check.py 2 2 --small > $O/graph_r06f_default.log 2>&1 && tail -n 2 $O/graph_r06f_default.log
