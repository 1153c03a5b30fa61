#!/bin/bash
# r06ax: the training forward's non-repeatable prediction with the loss targets beside it — where the join
# stops it (layers 14, 15), and whether it is an out-of-bounds store (RST_ALLOC_PAD guard bands around every trainer and
# loss-network buffer: canaries checked before every compute_gradients)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/race_r06ax.log
: > $O
for e in "RST_TARGETS_JOIN_AT=-1" "RST_TARGETS_JOIN_AT=14" "RST_TARGETS_JOIN_AT=15" \
         "RST_TARGETS_JOIN_AT=-1 RST_ALLOC_PAD=1048576"; do
    echo "== $e" >> $O
    env $e timeout -k 10 300 python -u tools/pred_race_check.py bf16 5 >> $O 2>&1 || { echo "rc=$?" >> $O; exit 1; }
done
cat $O
