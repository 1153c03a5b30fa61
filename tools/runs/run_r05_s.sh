#!/bin/bash
# round 5: residual-conv timelines with kernel arguments in device memory (as the graph replay has them), and the
# X6_SKIP knock-outs (1 no U reloads, 2 no transform, 4 no staging, 3, 7) of the accumulator-mode Cin-128 layer
# (the knock-outs fail the correctness gate by construction: only a time limit or a crash ends the script)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export HIP_FORCE_DEV_KERNARG=1
for b in prof_s2 prof_s4 prof_s3 prof_s7; do
  echo "== $b" >> gpurun_out/x6skip_r05s2.log
  timeout -k 10 120 tools/wino_x6_bench_$b 1 128 1 0 0 0 0 1 1 >> gpurun_out/x6skip_r05s2.log 2>&1
  rc=$?; [ $rc -ge 124 ] && exit $rc
done
grep -E "==|issue split|timeline|wino_x6 B" gpurun_out/x6skip_r05s2.log
