#!/bin/bash
# round 5: the style predictor's forward beside the transfer network's contract layers (rst_trainer_style_params_ready):
# training / predictor GPU tests, 3 same-box training-step pairs against RST_SERIAL_PREDICTOR_FWD=1, kernel trace
cd "$(dirname "$0")/../.."
TAG=r05ar bash tools/gpu_measure.sh "tests=train or predictor or distributed or checkpoint or keras" trainab=RST_SERIAL_PREDICTOR_FWD=1@-@3 trainprof
