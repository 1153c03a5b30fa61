#!/bin/bash
# r06bl: the last conv on scalar FMAs as the product form — the GPU suite, the targets race without a join on it
# (10 calls, dumps compared), and the config-4 step against the packed form (tools/var_pk.so), both with the join, 3 pairs
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/rdump
TAG=r06bl bash tools/gpu_measure.sh tests || exit 1
O=gpurun_out/race_r06bl.log
RST_TARGETS_JOIN_AT=-1 RST_RACE_DUMP=/tmp/rdump/d timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 > $O 2>&1 && \
python tools/race_dump_compare.py /tmp/rdump/d 10 480 960 >> $O 2>&1 || { echo "rc=$?"; cat $O; exit 1; }
grep "^call [0-9]: in" $O
TAG=r06bl bash tools/gpu_measure.sh "trainab=-@RST_LIB=tools/var_pk.so@3"
