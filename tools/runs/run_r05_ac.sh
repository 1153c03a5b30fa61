#!/bin/bash
# round 5: static priority (s_setprio 1) for the residual conv's second-dispatched wave half in the chunk loop:
# in-frame timelines both ways, then alternating headline pairs (a = library, b = variant)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in prof_librst prof_librst_prio; do
  echo "== $v" >> gpurun_out/frame_tl_r05ac.log
  RST_LIB=tools/$v.so timeout -k 10 300 python -u tools/frame_timeline.py 300 >> gpurun_out/frame_tl_r05ac.log 2>&1 || { tail -20 gpurun_out/frame_tl_r05ac.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/frame_tl_r05ac.log
TAG=r05ac bash tools/gpu_measure.sh ab=-@RST_LIB=tools/var_prio.so@3
