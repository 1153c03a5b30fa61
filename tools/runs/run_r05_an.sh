#!/bin/bash
# round 5: the style predictor's backward on a side stream from the point where grad_style_params is final
# (rst_trainer_wait_style_gradient): training / predictor / distributed GPU tests, 3 same-box training-step pairs against
# RST_SERIAL_PREDICTOR_BWD=1, and a kernel trace of the step
cd "$(dirname "$0")/../.."
TAG=r05an bash tools/gpu_measure.sh "tests=train or predictor or distributed or checkpoint or keras" trainab=RST_SERIAL_PREDICTOR_BWD=1@-@3 trainprof
