#!/bin/bash
# r06ba: the targets-beside-forward race bisected by kernel inside the last layer: join before forward kernel k
# (RST_TARGETS_JOIN_KERNEL; no layer join), 10 calls each
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/race_r06ba.log
: > $O
for k in 29 30 31 32 33 34; do
    echo "== RST_TARGETS_JOIN_AT=-1 RST_TARGETS_JOIN_KERNEL=$k" >> $O
    RST_TARGETS_JOIN_AT=-1 RST_TARGETS_JOIN_KERNEL=$k timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 >> $O 2>&1 \
        || { echo "rc=$?" >> $O; exit 1; }
done
cat $O
