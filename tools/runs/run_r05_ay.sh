#!/bin/bash
# round 5: the predictor's forward (the step's critical start) against the loss targets' VGG16 convs on the side
# stream: high-priority predictor-forward stream (RST_PFWD_HIPRIO=1) and targets queued after it (RST_TARGETS_AFTER=1),
# each in 3 same-box pairs against the default order
cd "$(dirname "$0")/../.."
TAG=r05ay bash tools/gpu_measure.sh "tests=beside or joint" trainab=-@RST_PFWD_HIPRIO=1@3 && \
TAG=r05ay2 bash tools/gpu_measure.sh trainab=-@RST_TARGETS_AFTER=1@3
