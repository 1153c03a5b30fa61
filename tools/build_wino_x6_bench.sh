#!/bin/bash
# Build tools/wino_x6_bench (gfx950) from the library's kernel sources.
set -e
cd "$(dirname "$0")/.."
F="$X6FLAGS -O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc"
mkdir -p /tmp/wx6b
/opt/rocm/bin/hipcc $F -c realtime_style_transfer_amd/csrc/wino.hip -o /tmp/wx6b/wino.o &
/opt/rocm/bin/hipcc $F -c ${X6SLP:--fno-slp-vectorize} realtime_style_transfer_amd/csrc/wino_x6.hip -o /tmp/wx6b/wino_x6.o &
/opt/rocm/bin/hipcc $F -c realtime_style_transfer_amd/csrc/norm.hip -o /tmp/wx6b/norm.o &
/opt/rocm/bin/hipcc $F -c tools/wino_x6_bench.hip -o /tmp/wx6b/main.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/wx6b/wino.o /tmp/wx6b/wino_x6.o /tmp/wx6b/norm.o /tmp/wx6b/main.o \
    -o tools/wino_x6_bench${X6SUFFIX}
