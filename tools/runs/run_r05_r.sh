#!/bin/bash
# round 5 (session 3): baseline of the restored tree: GPU suite, smoke, headline, kernel trace, residual timeline;
# HIP_FORCE_DEV_KERNARG=1 vs default headline pairs
cd "$(dirname "$0")/../.."
TAG=r05r bash tools/gpu_measure.sh tests smoke short prof x6prof=1,128,1,0,0,0,0,1,1 ab=HIP_FORCE_DEV_KERNARG=1@-@2
