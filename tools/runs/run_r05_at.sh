#!/bin/bash
# round 5: whole-tree validation of the final build: every GPU test, smoke, the default bench line, the headline's
# kernel trace and the training step's kernel trace
cd "$(dirname "$0")/../.."
TAG=r05at PYTEST_X=" " bash tools/gpu_measure.sh tests smoke bench prof trainprof
