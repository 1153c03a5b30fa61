#!/bin/bash
# r06b: GPU suite (bf16 VGG activations, timeline, fused start-conv tail), short bench (in-graph roofline), rocprof
# trace of it, headline A/B of the fused tail, training A/B of the bf16 activation storage
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06b bash tools/gpu_measure.sh tests short prof ab=RST_F3_FUSED_TAIL=0@-@3 trainab=RST_VGG_ACT_F32=1@-@3
