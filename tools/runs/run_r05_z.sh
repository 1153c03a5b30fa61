#!/bin/bash
# round 5: VGG16 conv layers, conv_bf3 production tiles vs conv_vgg.hip (two-stage prefetch), forward and dgrad
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/vgg_bench 4 0 > gpurun_out/vgg_bench_r05z.log 2>&1 && timeout -k 10 120 tools/vgg_bench 4 1 >> gpurun_out/vgg_bench_r05z.log 2>&1 || { tail -20 gpurun_out/vgg_bench_r05z.log; exit 1; }
cat gpurun_out/vgg_bench_r05z.log
TAG=r05z bash tools/gpu_measure.sh "tests=vgg_kernel"
