#!/bin/bash
# round 5: the trainer's re-pack gathers in batched launches: training GPU tests, 3 same-box training-step pairs
# against the previous build (tools/var_prevgather.so), kernel trace of the step
cd "$(dirname "$0")/../.."
TAG=r05au bash tools/gpu_measure.sh "tests=train or predictor or checkpoint or keras" trainab=RST_LIB=tools/var_prevgather.so@-@3 trainprof
