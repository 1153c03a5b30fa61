#!/bin/bash
# round 5: whole-tree validation after the late materialised stores: every GPU test, smoke, the default bench line and
# the kernel trace of the headline
cd "$(dirname "$0")/../.."
TAG=r05al PYTEST_X=" " bash tools/gpu_measure.sh tests smoke bench prof
