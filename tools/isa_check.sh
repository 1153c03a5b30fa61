#!/bin/bash
# Device-ISA check of csrc sources (CPU, no GPU): compile each with --save-temps into /tmp/isa and report per
# kernel VGPR/AGPR counts, spills and scratch, and fail if any scalar-memory store / atomic / cache write-back
# instruction appears (not allowed on the GPU pool).   Usage: bash tools/isa_check.sh wino_x6 conv_lite ...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p /tmp/isa
bad=0
for src in "$@"; do
    ( cd /tmp/isa && /opt/rocm/lib/llvm/bin/clang++ --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I /root/repo/include \
        -I /root/repo/realtime_style_transfer_amd/csrc -munsafe-fp-atomics $(python3 -c "import sys; sys.path.insert(0,'/root/repo'); from realtime_style_transfer_amd import build; print(' '.join(build.EXTRA.get('$src.hip', [])))" 2>/dev/null) \
        --save-temps -c -x hip /root/repo/realtime_style_transfer_amd/csrc/$src.hip -o $src.o 2>/dev/null ) || { echo "$src: compile failed"; exit 1; }
    s=/tmp/isa/$src-hip-amdgcn-amd-amdhsa-gfx950.s
    python3 - "$s" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)\.vgpr_spill_count:\s+(\d+)', txt, re.S):
    pass
names = re.findall(r'^\s+\.name:\s+(\S+)$', txt, re.M)
for k in re.finditer(r'- \.agpr_count:\s+(\d+).*?\.name:\s+(\S+).*?\.private_segment_fixed_size:\s+(\d+).*?\.sgpr_spill_count:\s+(\d+).*?\.vgpr_count:\s+(\d+)\n\s+\.vgpr_spill_count:\s+(\d+)', txt, re.S):
    agpr, name, scratch, sspill, vgpr, vspill = k.groups()
    flag = "  <-- SPILL/SCRATCH" if int(vspill) or int(scratch) else ""
    print(f"  {name[:90]:90s} v{vgpr} a{agpr} vspill {vspill} scratch {scratch}{flag}")
PY
    if grep -nE '^\s+(s_store|s_buffer_store|s_atomic|s_buffer_atomic|s_dcache_wb|s_dcache_discard|s_scratch_store)' "$s" >/dev/null; then
        echo "$src: SCALAR MEMORY WRITE INSTRUCTIONS FOUND"; bad=1
    fi
done
exit $bad
