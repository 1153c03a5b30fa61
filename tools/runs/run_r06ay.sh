#!/bin/bash
# r06ay: does any kernel of the training forward read LDS it did not write? The prediction with every CU's LDS filled
# with a pattern before each forward kernel (RST_LDS_POISON: quiet NaN, 1.0) against the plain one (targets joined
# before the forward, the repeatable configuration)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/poison_r06ay.log
: > $O
run() { echo "== $1" >> $O; env $1 timeout -k 10 300 python -u tools/pred_race_check.py bf16 2 1 gpurun_out/pred_$2.npy >> $O 2>&1; }
run "RST_TARGETS_JOIN_AT=0" plain && run "RST_LDS_POISON=0x7FC00000" nan && run "RST_LDS_POISON=0x3F800000" one || { echo "rc=$?" >> $O; cat $O; exit 1; }
python - >> $O 2>&1 <<'PY'
import numpy as np
a = np.load("gpurun_out/pred_plain.npy")
for k in ("nan", "one"):
    b = np.load(f"gpurun_out/pred_{k}.npy")
    d = np.abs(b.astype(np.float64) - a)
    print(f"{k}: NaN {int(np.isnan(b).sum())}, max |diff| {np.nanmax(d):.3e}, pixels differing "
          f"{int((np.nan_to_num(d, nan=1.0).reshape(a.shape[0], -1, 3).max(-1) > 0).sum())}")
PY
rm -f gpurun_out/pred_*.npy
cat $O
