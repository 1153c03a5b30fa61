#!/bin/bash
# round 5: full GPU suite + smoke + default bench line + kernel trace of the tree with the F(3x3) start conv
cd "$(dirname "$0")/../.."
TAG=r05j bash tools/gpu_measure.sh tests smoke bench prof
