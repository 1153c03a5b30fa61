#!/bin/bash
# round 5: the predictor-backward stream at high priority (own hardware queue); weight gradients beside the chain
# (default) against RST_SERIAL_WGRAD=1, 3 same-box pairs, then a kernel trace
cd "$(dirname "$0")/../.."
TAG=r05ap bash tools/gpu_measure.sh "tests=beside or joint" trainab=RST_SERIAL_WGRAD=1@-@3 trainprof
