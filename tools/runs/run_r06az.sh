#!/bin/bash
# r06az: more calls per setting for the targets-beside-forward race — no join, join before layer 15 (expand_last), and
# no join with the loss network's write-through stores off (RST_LOSS_WT=0)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/race_r06az.log
: > $O
for e in "RST_TARGETS_JOIN_AT=-1" "RST_TARGETS_JOIN_AT=15" "RST_TARGETS_JOIN_AT=-1 RST_LOSS_WT=0"; do
    echo "== $e" >> $O
    env $e timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 >> $O 2>&1 || { echo "rc=$?" >> $O; exit 1; }
done
cat $O
