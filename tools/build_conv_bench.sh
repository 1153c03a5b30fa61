#!/bin/bash
# Build the standalone conv micro-benchmark (gfx950).
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc tools/conv_bench.hip -o tools/conv_bench
