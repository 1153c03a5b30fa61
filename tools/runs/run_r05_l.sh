#!/bin/bash
# round 5: does the kernel-argument placement matter? headline with HIP_FORCE_DEV_KERNARG=1 vs default, same box;
# residual-conv timelines both ways
cd "$(dirname "$0")/../.."
TAG=r05l bash tools/gpu_measure.sh ab=HIP_FORCE_DEV_KERNARG=1@-@3 x6prof=1,128,1,0,0,0,0,1,1
HIP_FORCE_DEV_KERNARG=1 TAG=r05l2 bash tools/gpu_measure.sh x6prof=1,128,1,0,0,0,0,1,1
