#!/bin/bash
# round 5: helper materialisation with sixteen items in flight per thread: 3 same-box headline pairs vs in-loop stores
cd "$(dirname "$0")/../.."
TAG=r05aj bash tools/gpu_measure.sh ab=RST_X6_MAT_HELPERS=0@-@3
