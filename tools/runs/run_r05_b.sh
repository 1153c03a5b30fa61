#!/bin/bash
# round 5: the CIN affine with its accumulator loads unserialized and issued ahead of the staging loads
# (kernels.h CinAffineSplit), dead knobs removed, wgrad9_x6 alignment + split count. GPU suite, residual-conv timelines,
# same-box A/B of the headline against the round-4 library, kernel trace.
cd "$(dirname "$0")/../.."
TAG=r05b bash tools/gpu_measure.sh tests \
  x6prof=1,128,1,0,0,0,0,1,1 x6prof=1,128,3,0,0,0,0,0,1 \
  ab=RST_LIB=tools/librst_r04.so@-@3 prof
