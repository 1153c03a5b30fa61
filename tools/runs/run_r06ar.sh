#!/bin/bash
# r06ar: the bench's training leg measured after all side legs (bench_old_tmp.py, the previous order) against right after
# the headline (bench.py), twice each alternating; the new expand_0 two-forms GPU test
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transfer.py -m gpu -v --timeout 300 --timeout-method thread \
    -k expand0_ksplit > $O/pytest_r06ar.log 2>&1; echo "test rc=$?"; tail -3 $O/pytest_r06ar.log
for i in 1 2; do
  for b in bench_old_tmp.py bench.py; do
    timeout -k 10 600 python -u $b --no-cpu-baseline --train-modes bf16 > $O/order_r06ar_${b%.py}_$i.log 2>&1 || { tail -20 $O/order_r06ar_${b%.py}_$i.log; exit 1; }
    echo "$b run $i: $(grep -o '"value": [0-9.]*' $O/order_r06ar_${b%.py}_$i.log | head -1) training $(grep -o '"training": {.\{0,420\}' $O/order_r06ar_${b%.py}_$i.log | grep -o '"ms_per_step": [0-9.]*')"
  done
done
