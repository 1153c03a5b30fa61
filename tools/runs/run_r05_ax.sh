#!/bin/bash
# round 5: final whole-tree validation (after the batched re-pack gathers): every GPU test, smoke, the default bench
# line, the headline's kernel trace
cd "$(dirname "$0")/../.."
TAG=r05ax PYTEST_X=" " bash tools/gpu_measure.sh tests smoke bench prof
