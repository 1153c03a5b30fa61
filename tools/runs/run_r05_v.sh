#!/bin/bash
# round 5: idle-CU input prefetch for the residual convs (RST_X6_PREFETCH): in-frame timeline both ways, headline pairs,
# kernel trace, residual/transfer parity tests
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for pf in 0 1; do
  echo "== RST_X6_PREFETCH=$pf" >> gpurun_out/frame_tl_r05v.log
  RST_X6_PREFETCH=$pf RST_LIB=tools/prof_librst.so timeout -k 10 300 python -u tools/frame_timeline.py 300 >> gpurun_out/frame_tl_r05v.log 2>&1 || { tail -20 gpurun_out/frame_tl_r05v.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/frame_tl_r05v.log
TAG=r05v bash tools/gpu_measure.sh "tests=transfer or winograd or residual" ab=RST_X6_PREFETCH=0@-@3 prof
