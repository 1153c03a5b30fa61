#!/bin/bash
# r06be: what differs when the race hits — the last layer's input, raw output and statistics partials per call
# (RST_RACE_DUMP), no join, 10 calls
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/rdump
O=gpurun_out/race_r06be.log
RST_TARGETS_JOIN_AT=-1 RST_RACE_DUMP=/tmp/rdump/d timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 > $O 2>&1 && \
python tools/race_dump_compare.py /tmp/rdump/d 10 480 960 >> $O 2>&1; echo "rc=$?" >> $O
cat $O
