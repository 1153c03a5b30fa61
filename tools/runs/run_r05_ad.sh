#!/bin/bash
# round 5: validation of the tree: GPU suite, smoke, default bench line, frame kernel trace
cd "$(dirname "$0")/../.."
TAG=r05ad bash tools/gpu_measure.sh tests smoke bench prof
