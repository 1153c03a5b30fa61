#!/bin/bash
# round 5: the materialised-output stores issued after the chunk's last U / staging loads (X6_MAT_LATE=1, this build)
# against the in-place stores (tools/var_matearly.so): GPU tests, in-frame timelines of forms 2 and 3, 3 headline pairs
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=gpurun_out/frame_tl_matlate_r05ak.log
for v in p2 p3; do
  echo "== $v" >> $L
  RST_LIB=tools/prof_librst_$v.so timeout -k 10 240 python tools/frame_timeline.py 300 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
cat $L
TAG=r05ak bash tools/gpu_measure.sh "tests=transfer or configs or layer or two_style" ab=RST_LIB=tools/var_matearly.so@-@3
