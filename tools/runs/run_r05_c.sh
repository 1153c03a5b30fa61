#!/bin/bash
# round 5: conv_lite x6 single-chunk layers back to 2 waves/SIMD (lean CIN affine form); config-4 parity at scale
# against the f32 oracle; same-box A/B of the headline against the round-4 library; kernel trace.
cd "$(dirname "$0")/../.."
TAG=r05c bash tools/gpu_measure.sh tests=at_scale ab=RST_LIB=tools/librst_r04.so@-@3 prof
