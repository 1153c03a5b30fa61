#!/bin/bash
# r06b: GPU suite (bf16 VGG activations, timeline), short bench (in-graph roofline), rocprof trace of it, training A/B
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06b bash tools/gpu_measure.sh tests short prof trainab=RST_VGG_ACT_F32=1@-@3
