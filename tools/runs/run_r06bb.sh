#!/bin/bash
# r06bb: is the race a visibility problem at a kernel boundary or inside the last conv? A barrier packet (event from an
# idle stream, RST_FENCE_KERNEL) before the last conv / before its finalize, with the targets joined before the
# finalize or not at all; 10 calls each
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/race_r06bb.log
: > $O
for e in "RST_TARGETS_JOIN_KERNEL=32 RST_FENCE_KERNEL=31" "RST_FENCE_KERNEL=31" "RST_FENCE_KERNEL=32" "RST_FENCE_KERNEL=33"; do
    echo "== RST_TARGETS_JOIN_AT=-1 $e" >> $O
    env RST_TARGETS_JOIN_AT=-1 $e timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 >> $O 2>&1 \
        || { echo "rc=$?" >> $O; exit 1; }
done
cat $O
