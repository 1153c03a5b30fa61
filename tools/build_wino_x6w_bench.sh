#!/bin/bash
# Build tools/wino_x6w_bench (gfx950) from the library's kernel sources.
set -e
cd "$(dirname "$0")/.."
F="$X6FLAGS -O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc"
mkdir -p /tmp/wx6wb
/opt/rocm/bin/hipcc $F -c realtime_style_transfer_amd/csrc/wino.hip -o /tmp/wx6wb/wino.o &
/opt/rocm/bin/hipcc $F -c -fno-slp-vectorize realtime_style_transfer_amd/csrc/wino_x6.hip -o /tmp/wx6wb/wino_x6.o &
/opt/rocm/bin/hipcc $F -c -fno-slp-vectorize tools/wino_x6w.hip -o /tmp/wx6wb/wino_x6w.o &
/opt/rocm/bin/hipcc $F -c tools/wino_x6w_bench.hip -o /tmp/wx6wb/main.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/wx6wb/wino.o /tmp/wx6wb/wino_x6.o /tmp/wx6wb/wino_x6w.o /tmp/wx6wb/main.o \
    -o tools/wino_x6w_bench${X6SUFFIX}
