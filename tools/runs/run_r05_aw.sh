#!/bin/bash
# round 5: BatchNorm backward finalize inside the apply for few-partial layers (predictor training): predictor /
# training GPU tests, 3 same-box training-step pairs against RST_BN_BWD_FUSE=0, kernel trace
cd "$(dirname "$0")/../.."
TAG=r05aw bash tools/gpu_measure.sh "tests=train or predictor or checkpoint or keras" trainab=RST_BN_BWD_FUSE=0@-@3 trainprof
