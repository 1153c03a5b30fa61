#!/bin/bash
# round 5: start conv on F(3x3, 3x3) tiles (wino9f3.hip). Parity of the start conv and the full network first; then the
# headline against the round-4 library and against RST_START_F3=0 on the same box, kernel trace.
cd "$(dirname "$0")/../.."
TAG=r05d PYTEST_X=-x bash tools/gpu_measure.sh "tests=start_conv_f3 or winograd or at_scale" short \
  ab=RST_START_F3=0@-@2 prof
