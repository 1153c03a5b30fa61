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
    # accumulator modes change the prologue's affine source, so the f32-vs-x6 self check reports a mismatch
    # (exit 1): only a time limit or a crash stops the loop
    timeout -k 5 60 tools/wino_x6_bench_v4 $args >> gpurun_out/x6acc.log 2>&1
    rc=$?
    if [ $rc -ge 124 ]; then tail -20 gpurun_out/x6acc.log; exit 1; fi
done
grep "==\|wino_x6 B" gpurun_out/x6acc.log
