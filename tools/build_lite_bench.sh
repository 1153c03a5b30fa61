#!/bin/bash
# Build the standalone narrow-conv micro-benchmark (gfx950). LITEFLAGS: extra -D knobs; LITESUFFIX: binary suffix.
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 ${LITEFLAGS} -I include -I realtime_style_transfer_amd/csrc \
    tools/lite_bench.hip -o tools/lite_bench${LITESUFFIX}
