#!/bin/bash
# r03: conv_bf3 two-stage weight prefetch (config 136 and variants) on the VGG16 layers (tools/conv_bench 4 vgg),
# loss/train GPU tests of the refactored stage loop.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 tools/conv_bench 4 vgg > gpurun_out/conv_bench_vgg_z.log 2>&1 || { tail -20 gpurun_out/conv_bench_vgg_z.log; exit 1; }
cat gpurun_out/conv_bench_vgg_z.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_z.log 2>&1 || { tail -40 gpurun_out/pytest_z.log; exit 1; }
tail -1 gpurun_out/pytest_z.log
