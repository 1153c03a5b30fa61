#!/bin/bash
# Build tools/wino9f3_bench (gfx950) from the library's kernel sources ($F3FLAGS: experiment -D flags, $F3SUFFIX).
set -e
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc"
D=/tmp/f3b$$
mkdir -p $D
/opt/rocm/bin/hipcc $F -c realtime_style_transfer_amd/csrc/wino9.hip -o $D/wino9.o &
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -c realtime_style_transfer_amd/csrc/wino9_x6.hip -o $D/wino9_x6.o &
/opt/rocm/bin/hipcc $F $F3FLAGS -c realtime_style_transfer_amd/csrc/wino9f3.hip -o $D/wino9f3.o &
/opt/rocm/bin/hipcc $F $F3FLAGS -c tools/wino9f3_bench.hip -o $D/main.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 $D/wino9.o $D/wino9_x6.o $D/wino9f3.o $D/main.o -o tools/wino9f3_bench${F3SUFFIX}
rm -rf $D
