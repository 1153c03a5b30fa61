#!/bin/bash
# round 5: the frame's last residual conv timeline (hipGraph replay, profiling library)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
RST_LIB=tools/prof_librst.so timeout -k 10 300 python -u tools/frame_timeline.py 300 > gpurun_out/frame_tl_r05t.log 2>&1 || { tail -20 gpurun_out/frame_tl_r05t.log; exit 1; }
cat gpurun_out/frame_tl_r05t.log
