#!/bin/bash
# r06ai: re-run of the config-4 480x960 bf16-VGG parity test alone (failed once in r06ah with prediction 8.3e-3),
# then the whole training file, then config-4 step A/B pairs for the predictor BN merge (RST_BN_MERGE=0: launches)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
PYTEST_X=" " TAG=r06ai1 bash tools/gpu_measure.sh "tests=config4_480x960_bf16_vgg"
cp gpurun_out/train_parity_scale_full_bf16_winograd_bf16x6.json gpurun_out/r06ai1_full_bf16.json
PYTEST_X=" " TAG=r06ai2 bash tools/gpu_measure.sh "tests=test_gpu_train" || true
TAG=r06ai bash tools/gpu_measure.sh trainab=RST_BN_MERGE=0@-@3
