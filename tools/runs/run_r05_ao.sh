#!/bin/bash
# round 5: the transfer network's weight gradients on the trainer's side stream beside the input-gradient chain
# (norm-backward outputs in a ring of three buffers): training / predictor / distributed GPU tests, 3 same-box
# training-step pairs against RST_SERIAL_WGRAD=1, and a kernel trace of the step
cd "$(dirname "$0")/../.."
TAG=r05ao bash tools/gpu_measure.sh "tests=train or predictor or distributed or checkpoint or keras" trainab=RST_SERIAL_WGRAD=1@-@3 trainprof
