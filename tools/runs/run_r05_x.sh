#!/bin/bash
# round 5: VGG16 convs on conv_vgg.hip (8-wave 16x16 tile): loss / training parity tests, then the config-4 training
# step with the new kernel (default) against conv_bf3's tiles (RST_VGG_CONV=0), alternating on one box
cd "$(dirname "$0")/../.."
TAG=r05x bash tools/gpu_measure.sh "tests=vgg_kernel or style_loss or training_step_matches_oracle" trainab=RST_VGG_CONV=0@-@2
