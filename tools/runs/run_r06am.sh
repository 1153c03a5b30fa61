#!/bin/bash
# r06am: bisect the prediction race — the forward joins the loss targets before layer k (RST_TARGETS_JOIN_AT=k);
# bitwise-repeatable predictions from some k down mean the race is with layers >= that k
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
for k in 0 1 3 8 13 16; do
  echo "== RST_TARGETS_JOIN_AT=$k"
  RST_TARGETS_JOIN_AT=$k timeout -k 10 300 python -u tools/pred_race_check.py bf16 5 || exit 1
done 2>&1 | grep -v amdgpu.ids | tee $O/race_r06am.log
