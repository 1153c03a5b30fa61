#!/bin/bash
# Build tools/wino9_x6_bench (gfx950) from the library's kernel sources ($W9FLAGS: experiment -D flags).
set -e
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc"
D=/tmp/w9b$$
mkdir -p $D
/opt/rocm/bin/hipcc $F -c realtime_style_transfer_amd/csrc/wino9.hip -o $D/wino9.o &
/opt/rocm/bin/hipcc $F $W9FLAGS -fno-slp-vectorize -c realtime_style_transfer_amd/csrc/wino9_x6.hip -o $D/wino9_x6.o &
/opt/rocm/bin/hipcc $F $W9FLAGS -c tools/wino9_x6_bench.hip -o $D/main.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 $D/wino9.o $D/wino9_x6.o $D/main.o -o tools/wino9_x6_bench${W9SUFFIX}
rm -rf $D
