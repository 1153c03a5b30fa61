#!/bin/bash
# round 5, first box: GPU suite, headline + kernel trace of this round's starting tree, residual-conv timelines
# (accumulator mode with the correctness gate seeded from real statistics)
cd "$(dirname "$0")/../.."
TAG=r05a bash tools/gpu_measure.sh tests short prof \
  x6prof=1,128,1,0,0,0,0,1,1 x6prof=1,128,3,0,0,0,0,0,1 x6prof=1,32,0,0,0,0,0,0,2 \
  x6bench=1,128,1,0,0,0,0,1,1 x6bench=1,128,3,0,0,0,0,0,1
