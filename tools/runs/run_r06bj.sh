#!/bin/bash
# r06bj: the targets race with the last conv's packed FMAs replaced by scalar ones (tools/var_nopk.so, built with
# -DRST_SMALL_NOPK: no v_pk_fma_f32 in the kernel) against the product build; no join, 10 calls each, dumps compared
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/rdump
O=gpurun_out/race_r06bj.log
: > $O
for lib in tools/var_nopk.so realtime_style_transfer_amd/librst.so tools/var_nopk.so; do
    echo "== RST_TARGETS_JOIN_AT=-1 RST_LIB=$lib" >> $O
    rm -f /tmp/rdump/*
    RST_LIB=$lib RST_TARGETS_JOIN_AT=-1 RST_RACE_DUMP=/tmp/rdump/d timeout -k 10 300 python -u tools/pred_race_check.py bf16 10 \
        >> $O 2>&1 && python tools/race_dump_compare.py /tmp/rdump/d 10 480 960 >> $O 2>&1 || { echo "rc=$?" >> $O; cat $O; exit 1; }
done
cat $O
