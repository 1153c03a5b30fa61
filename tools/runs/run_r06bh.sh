#!/bin/bash
# r06bh: the differing last-conv outputs of the targets race, value by value (call 0 vs this call, bit patterns)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/rdump
O=gpurun_out/race_r06bh.log
: > $O
for e in "RST_SMALL_EXCLUSIVE=0"; do
    echo "== RST_TARGETS_JOIN_AT=-1 $e" >> $O
    rm -f /tmp/rdump/*
    env RST_TARGETS_JOIN_AT=-1 RST_RACE_DUMP=/tmp/rdump/d $e timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 >> $O 2>&1 && \
    python tools/race_dump_compare.py /tmp/rdump/d 10 480 960 >> $O 2>&1 || { echo "rc=$?" >> $O; cat $O; exit 1; }
done
cat $O
