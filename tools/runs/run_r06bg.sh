#!/bin/bash
# r06bg: (a) are the VGG16 targets themselves repeatable (targets joined, losses compared per call)? (b) does the last conv
# read LDS outside its arrays? Alone on its CU (RST_SMALL_EXCLUSIVE) with the rest of the LDS poisoned with NaN before
# it (RST_LDS_POISON, layer 15), against the plain prediction
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/race_r06bg.log
: > $O
echo "== RST_TARGETS_JOIN_AT=0" >> $O
RST_TARGETS_JOIN_AT=0 timeout -k 10 300 python -u tools/pred_race_check.py bf16 6 1 gpurun_out/pred_plain.npy >> $O 2>&1 && \
echo "== RST_SMALL_EXCLUSIVE=1 RST_LDS_POISON=0x7FC00000 RST_LDS_POISON_LAYER=15" >> $O && \
RST_SMALL_EXCLUSIVE=1 RST_LDS_POISON=0x7FC00000 RST_LDS_POISON_LAYER=15 timeout -k 10 300 python -u tools/pred_race_check.py \
    bf16 3 1 gpurun_out/pred_excl.npy >> $O 2>&1 || { echo "rc=$?" >> $O; cat $O; exit 1; }
python - >> $O 2>&1 <<'PY'
import numpy as np
a = np.load("gpurun_out/pred_plain.npy"); b = np.load("gpurun_out/pred_excl.npy")
d = np.abs(b.astype(np.float64) - a)
print(f"exclusive+poison vs plain: NaN {int(np.isnan(b).sum())}, max |diff| {np.nanmax(d):.3e}")
PY
rm -f gpurun_out/pred_*.npy
cat $O
