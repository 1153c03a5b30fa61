#!/bin/bash
# r06al: is the training forward's prediction repeatable with the bf16-VGG loss targets beside it? (tools/
# pred_race_check.py: default, RST_SERIAL_TARGETS=1, RST_TRAIN_WT=0); the training file in order with RST_TRAIN_WT=0;
# the tap-row residual weight gradient standalone with its own split count
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
for e in - RST_SERIAL_TARGETS=1 RST_TRAIN_WT=0; do
  echo "== $e"
  if [ "$e" = "-" ]; then timeout -k 10 300 python -u tools/pred_race_check.py bf16 6; else env $e timeout -k 10 300 python -u tools/pred_race_check.py bf16 6; fi
  echo "rc=$?"
done 2>&1 | tee $O/race_r06al.log
RST_TRAIN_WT=0 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k test_gpu_train \
     > $O/pytest_r06al_wt0.log 2>&1; echo "wt0 tests rc=$?"; tail -1 $O/pytest_r06al_wt0.log
timeout -k 10 120 tools/wgrad_r06al 4 > $O/wgrad_r06al_x6r.log 2>&1; echo "x6r rc=$?"; cat $O/wgrad_r06al_x6r.log
RST_WGRAD_X6R=0 timeout -k 10 120 tools/wgrad_r06al 4 > $O/wgrad_r06al_x6.log 2>&1; echo "x6 rc=$?"; cat $O/wgrad_r06al_x6.log
