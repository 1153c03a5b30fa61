#!/bin/bash
# Build tools/probe_r06 (gfx950): graph event timing, FETCH/WRITE_SIZE calibration, in-launch barrier vs boundary.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe_r06.hip -o tools/probe_r06
