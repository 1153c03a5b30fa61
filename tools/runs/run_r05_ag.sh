#!/bin/bash
# round 5: in-frame per-wave timelines of each residual-conv prologue form (X6_PROF_PRO = 1, 2, 3)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=gpurun_out/frame_tl_pro_r05ag.log
for p in 1 2 3; do
  echo "== PRO=$p" >> $L
  RST_LIB=tools/prof_librst_p$p.so timeout -k 10 240 python tools/frame_timeline.py 300 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
cat $L
