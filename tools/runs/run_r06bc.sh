#!/bin/bash
# r06bc: which part of the loss targets disturbs the last transfer conv beside it (RST_TARGETS_PARTS: 1 style VGG16,
# 2 its Grams, 4 content VGG16, 8 the content copy); no join; 10 calls each
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/race_r06bc.log
: > $O
for p in 15 1 3 4 12 7; do
    echo "== RST_TARGETS_JOIN_AT=-1 RST_TARGETS_PARTS=$p" >> $O
    RST_TARGETS_JOIN_AT=-1 RST_TARGETS_PARTS=$p timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 >> $O 2>&1 \
        || { echo "rc=$?" >> $O; exit 1; }
done
cat $O
