#!/bin/bash
# round 5: config-4 training-step kernel trace of the current tree
cd "$(dirname "$0")/../.."
TAG=r05p bash tools/gpu_measure.sh trainprof
