#!/bin/bash
# round 5: the predictor backward's weight gradients / outer products on a stream beside its input-gradient chain:
# training / predictor GPU tests, 3 same-box training-step pairs against RST_SERIAL_PREDICTOR_WGRAD=1, kernel trace
cd "$(dirname "$0")/../.."
TAG=r05aq bash tools/gpu_measure.sh "tests=train or predictor or distributed or checkpoint or keras" trainab=RST_SERIAL_PREDICTOR_WGRAD=1@-@3 trainprof
