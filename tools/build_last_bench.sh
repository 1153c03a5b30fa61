#!/bin/bash
# Build the final-layer micro-benchmark (gfx950). LASTFLAGS: extra -D knobs; LASTSUFFIX: binary suffix.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 ${LASTFLAGS} -I include -I realtime_style_transfer_amd/csrc \
    tools/last_bench.hip -o tools/last_bench${LASTSUFFIX}
