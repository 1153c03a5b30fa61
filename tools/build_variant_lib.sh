#!/bin/bash
# A variant of librst.so with some kernel sources rebuilt under extra flags, for same-box A/B runs (RST_LIB=...).
# Usage: VFLAGS="-DX6_PIN_ARGS" bash tools/build_variant_lib.sh NAME src1.hip [src2.hip ...]  -> tools/var_NAME.so
# (needs the library built first: python -m realtime_style_transfer_amd.build)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
D=/tmp/varlib$$
mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I realtime_style_transfer_amd/csrc -Wall -Wno-unused-function -Wno-unused-variable -munsafe-fp-atomics"
excl=""
for src in "$@"; do
  extra=""; case $src in wino_x6.hip|wino9_x6.hip|conv_small.hip) extra="-fno-slp-vectorize" ;; esac
  /opt/rocm/bin/hipcc $F $extra $VFLAGS -c realtime_style_transfer_amd/csrc/$src -o $D/${src%.hip}.o &
  excl="$excl|/${src%.hip}.o\$"
done
wait
objs=$(ls realtime_style_transfer_amd/_build/*.o | grep -Ev "${excl#|}")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs $D/*.o -o tools/var_$name.so
rm -rf $D
echo tools/var_$name.so
