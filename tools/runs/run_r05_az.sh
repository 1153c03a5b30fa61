#!/bin/bash
# round 5: with the late materialised stores, write-back (RST_WT_STORES=13) vs write-through (default 15) for them:
# 3 same-box headline pairs
cd "$(dirname "$0")/../.."
TAG=r05az bash tools/gpu_measure.sh ab=RST_WT_STORES=13@-@3
