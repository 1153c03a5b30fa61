#!/bin/bash
# r06ak: (1) the 480x960 bf16-VGG parity test after the training file's earlier tests, with the loss targets on the
# caller's stream (RST_SERIAL_TARGETS=1) and with f32 VGG16 activations (RST_VGG_ACT_F32=1) — which one cures the
# order-dependent prediction error; (2) the tap-row residual weight gradient standalone (tools/wgrad_bench:
# new kernel vs the x6 tile kernel vs f32)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
for e in RST_SERIAL_TARGETS=1 RST_VGG_ACT_F32=1; do
  env $e timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k test_gpu_train \
     > $O/pytest_r06ak_${e%%=*}.log 2>&1; echo "$e rc=$?"; tail -1 $O/pytest_r06ak_${e%%=*}.log
  grep -o '"prediction_max_abs": [0-9.e-]*' $O/train_parity_scale_full_bf16_winograd_bf16x6.json
done
timeout -k 10 120 tools/wgrad_r06ak 4 > $O/wgrad_r06ak_x6r.log 2>&1; echo "x6r rc=$?"; cat $O/wgrad_r06ak_x6r.log
RST_WGRAD_X6R=0 timeout -k 10 120 tools/wgrad_r06ak 4 > $O/wgrad_r06ak_x6.log 2>&1; echo "x6 rc=$?"; cat $O/wgrad_r06ak_x6.log
