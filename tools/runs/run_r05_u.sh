#!/bin/bash
# round 5: wino_x6 with every kernel argument pinned in SGPRs at the start (X6_PIN_ARGS): in-frame timeline of the last
# residual conv both ways, then alternating headline runs (a = library, b = pinned variant)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in prof_librst prof_librst_pin; do
  echo "== $v" >> gpurun_out/frame_tl_r05u.log
  RST_LIB=tools/$v.so timeout -k 10 300 python -u tools/frame_timeline.py 300 >> gpurun_out/frame_tl_r05u.log 2>&1 || { tail -20 gpurun_out/frame_tl_r05u.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/frame_tl_r05u.log
TAG=r05u bash tools/gpu_measure.sh ab=-@RST_LIB=tools/var_pin.so@3
