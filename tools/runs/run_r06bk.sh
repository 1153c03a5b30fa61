#!/bin/bash
# r06bk: what the fence costs — the config-4 training step with the scalar-FMA last conv and no targets join
# (tools/var_nopk.so, RST_TARGETS_JOIN_AT=-1) against the product (packed FMAs, join before layer 0), 3 pairs
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=r06bk bash tools/gpu_measure.sh "trainab=RST_LIB=tools/var_nopk.so:RST_TARGETS_JOIN_AT=-1@-@3"
