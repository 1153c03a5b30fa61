#!/bin/bash
# r03: where the residual conv's CIN-accumulator cost sits (standalone, B=1, Cin 128): partials + given affine,
# accumulators both ways, producer side only, consumer side only; ReLU and skip-add prologues.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rm -f gpurun_out/x6acc.log
for args in "1 128 1 0 0 0 0 1 0" "1 128 1 0 0 0 0 1 1" "1 128 1 0 0 0 0 1 2" "1 128 1 0 0 0 0 1 3" \
            "1 128 3 0 0 0 0 0 0" "1 128 3 0 0 0 0 0 1" "1 128 1 0 0 0 0 1 0" "1 128 1 0 0 0 0 1 1"; do
    echo "== $args" >> gpurun_out/x6acc.log
    timeout -k 5 60 tools/wino_x6_bench_v4 $args >> gpurun_out/x6acc.log 2>&1 || { tail -20 gpurun_out/x6acc.log; exit 1; }
done
grep "==\|wino_x6 B" gpurun_out/x6acc.log
