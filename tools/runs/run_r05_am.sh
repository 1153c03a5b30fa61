#!/bin/bash
# round 5: kernel trace of the config-4 training step (per-dispatch start/end for the step's stream overlap analysis)
cd "$(dirname "$0")/../.."
TAG=r05am bash tools/gpu_measure.sh trainprof
