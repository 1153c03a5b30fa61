#!/bin/bash
# r03: narrow-conv standalone timings (x6 expand_0 form), base vs the halo two steps ahead for multi-chunk
# layers (LITE_HPF2), and the base per-step timeline (LITE_PROF).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
{ for r in 1 2; do echo "== base"; timeout -k 10 120 tools/lite_bench_x6 200; echo "== HPF2"; timeout -k 10 120 tools/lite_bench_x6h 200; done
  echo "== LITE_PROF"; timeout -k 10 120 tools/lite_bench_x6p 50; } > gpurun_out/lite_h.log 2>&1
cat gpurun_out/lite_h.log
