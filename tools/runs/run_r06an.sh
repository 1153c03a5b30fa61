#!/bin/bash
# r06an: the forward joins the loss targets first (default now) — prediction repeatability, the training file in order,
# config-4 step pairs against the old overlap (RST_TARGETS_JOIN_AT=-1); the tap-row weight gradient with balanced,
# split-once staging standalone
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u tools/pred_race_check.py bf16 5 2>&1 | grep -v amdgpu.ids | tee $O/race_r06an.log || exit 1
timeout -k 10 120 tools/wgrad_r06an 4 > $O/wgrad_r06an_x6r.log 2>&1; echo "x6r rc=$?"; cat $O/wgrad_r06an_x6r.log
PYTEST_X=" " TAG=r06an bash tools/gpu_measure.sh "tests=test_gpu_train" || exit 1
TAG=r06an bash tools/gpu_measure.sh trainab=RST_TARGETS_JOIN_AT=-1@-@2
