#!/bin/bash
# A profiling variant of librst.so (tools/prof_librst.so): the library's objects with wino_x6.hip rebuilt under
# -DX6_PROF (per-wave timeline stamps; rst_debug_x6_timeline prints the last launch's). Run the frame with
# RST_LIB=tools/prof_librst.so python tools/frame_timeline.py. Needs the library built first (python -m
# realtime_style_transfer_amd.build).
set -e
cd "$(dirname "$0")/.."
D=/tmp/proflib$$
mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DX6_PROF=256 $PROFFLAGS -c realtime_style_transfer_amd/csrc/wino_x6.hip -o $D/wino_x6.o
objs=$(ls realtime_style_transfer_amd/_build/*.o | grep -v '/wino_x6.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs $D/wino_x6.o -o tools/prof_librst${PROFSUFFIX}.so
rm -rf $D
