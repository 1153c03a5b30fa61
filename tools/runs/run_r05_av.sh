#!/bin/bash
# round 5: the predictor backward's dz ring 3 -> 8 buffers (the chain stalled on slot releases): predictor / training
# GPU tests, 3 same-box training-step pairs against the ring-3 build (tools/var_dzr3.so), kernel trace
cd "$(dirname "$0")/../.."
TAG=r05av bash tools/gpu_measure.sh "tests=beside or joint or predictor" trainab=RST_LIB=tools/var_dzr3.so@-@3 trainprof
