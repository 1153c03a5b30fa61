#!/bin/bash
# r06bf: the last conv alone on its CUs (RST_SMALL_EXCLUSIVE: its workgroup takes the whole LDS) beside the targets,
# then the same without; the last layer's dumps compared per call (RST_RACE_DUMP), no join, 10 calls each
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/rdump
O=gpurun_out/race_r06bf.log
: > $O
for e in "RST_SMALL_EXCLUSIVE=1" "RST_SMALL_EXCLUSIVE=0"; do
    echo "== RST_TARGETS_JOIN_AT=-1 $e" >> $O
    rm -f /tmp/rdump/*
    env RST_TARGETS_JOIN_AT=-1 RST_RACE_DUMP=/tmp/rdump/d $e timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 >> $O 2>&1 && \
    python tools/race_dump_compare.py /tmp/rdump/d 10 480 960 >> $O 2>&1 || { echo "rc=$?" >> $O; cat $O; exit 1; }
done
cat $O
