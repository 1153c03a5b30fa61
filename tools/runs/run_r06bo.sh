#!/bin/bash
# r06bo: the inference path under co-residency — two full-size networks on two streams at once, 20 rounds, bitwise
# against each network alone
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/concurrent_infer_check.py 20 > gpurun_out/conc_r06bo.log 2>&1; echo "rc=$?" >> gpurun_out/conc_r06bo.log
cat gpurun_out/conc_r06bo.log
