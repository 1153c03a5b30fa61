#!/bin/bash
# Build tools/icache_x6 (gfx950) from the library's residual-conv source.
set -e
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc"
mkdir -p /tmp/icx6
/opt/rocm/bin/hipcc $F -c -fno-slp-vectorize realtime_style_transfer_amd/csrc/wino_x6.hip -o /tmp/icx6/wino_x6.o &
/opt/rocm/bin/hipcc $F -c realtime_style_transfer_amd/csrc/wino.hip -o /tmp/icx6/wino.o &
/opt/rocm/bin/hipcc $F -c tools/icache_x6.hip -o /tmp/icx6/main.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/icx6/wino_x6.o /tmp/icx6/wino.o /tmp/icx6/main.o -o tools/icache_x6
