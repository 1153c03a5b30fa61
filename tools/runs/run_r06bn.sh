#!/bin/bash
# r06bn: the final build without the targets join at the config-4 batch (B = 4), 10 calls, dumps compared
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/rdump
O=gpurun_out/race_r06bn.log
RST_TARGETS_JOIN_AT=-1 RST_RACE_DUMP=/tmp/rdump/d timeout -k 10 400 python -u tools/pred_race_check.py bf16 10 4 > $O 2>&1 && \
python tools/race_dump_compare.py /tmp/rdump/d 10 480 960 >> $O 2>&1; echo "rc=$?" >> $O
cat $O
