#!/bin/bash
# round 5: the materialised block output stored by the idle-CU helper workgroups (RST_X6_MAT_HELPERS, default on):
# transfer / configs GPU tests (bitwise batched-vs-per-frame covers helpers vs in-loop stores), in-frame timelines of
# prologue forms 2 and 3, then 3 same-box headline pairs against RST_X6_MAT_HELPERS=0
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=gpurun_out/frame_tl_mathelp_r05ai.log
for v in p2 p3; do
  echo "== $v" >> $L
  RST_LIB=tools/prof_librst_$v.so timeout -k 10 240 python tools/frame_timeline.py 300 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
cat $L
TAG=r05ai bash tools/gpu_measure.sh "tests=transfer or configs or layer or two_style" ab=RST_X6_MAT_HELPERS=0@-@3
