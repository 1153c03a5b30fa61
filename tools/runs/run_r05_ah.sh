#!/bin/bash
# round 5: knock-out — the materialised block output stores of the residual convs' prologue forms 2 / 3 removed
# (X6_SKIP bit 4; outputs wrong, timing only), in-frame timelines against the normal forms
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=gpurun_out/frame_tl_nomat_r05ah.log
for v in p2 p2nomat p3 p3nomat; do
  echo "== $v" >> $L
  RST_LIB=tools/prof_librst_$v.so timeout -k 10 240 python tools/frame_timeline.py 300 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
cat $L
