#!/bin/bash
# r06ap: tap-row weight gradient with the split's VALU interleaved between the MFMAs (sched_group_barrier, 2 or 3 VALU
# per MFMA) against the plain order; the frame's kernel trace on the current build (expand_0 K split in the frame)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
for v in 0 2 3 0 2 3; do
  timeout -k 10 120 tools/wx6r_ap_$v 4 > $O/wgrad_r06ap_$v.log 2>&1 || { cat $O/wgrad_r06ap_$v.log; exit 1; }
  echo "interleave $v: $(grep wgrad_x6 $O/wgrad_r06ap_$v.log) $(grep relative $O/wgrad_r06ap_$v.log | grep -o 'relative [0-9.e-]*')"
done
TAG=r06ap bash tools/gpu_measure.sh prof
