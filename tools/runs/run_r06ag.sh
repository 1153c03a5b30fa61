#!/bin/bash
# r06ag: expand_0's K split (8 waves, LDS-DMA weights) — standalone bench + timeline against the four-wave form,
# the GPU suite, then headline A/B pairs (RST_LITE_KSPLIT=0 restores the four-wave form)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 120 tools/lite_r06ag 200 > $O/lite_r06ag_ksplit.log 2>&1 || { tail -30 $O/lite_r06ag_ksplit.log; exit 1; }
cat $O/lite_r06ag_ksplit.log
RST_LITE_KSPLIT=0 timeout -k 10 120 tools/lite_r06ag 200 > $O/lite_r06ag_four.log 2>&1 || { tail -30 $O/lite_r06ag_four.log; exit 1; }
cat $O/lite_r06ag_four.log
timeout -k 10 120 tools/lite_r06ag_prof 20 > $O/liteprof_r06ag_ksplit.log 2>&1 || { tail -30 $O/liteprof_r06ag_ksplit.log; exit 1; }
RST_LITE_KSPLIT=0 timeout -k 10 120 tools/lite_r06ag_prof 20 > $O/liteprof_r06ag_four.log 2>&1 || { tail -30 $O/liteprof_r06ag_four.log; exit 1; }
TAG=r06ag bash tools/gpu_measure.sh tests || exit 1
TAG=r06ag bash tools/gpu_measure.sh ab=RST_LITE_KSPLIT=0@-@3
