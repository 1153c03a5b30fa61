# r04 call 9: x6 transposed-conv output staged through LDS (whole-line 16-B stores) vs per-accumulator stores,
# standalone and checked; GPU tests; residual convs' accumulator copies 2 and 1 vs 4
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do for v in x6 x6nost; do echo "== $v"; timeout -k 10 120 ./tools/lite_bench_$v 200 || exit 1; done; done
  echo "== x6prof"; timeout -k 10 120 ./tools/lite_bench_x6prof 50 || exit 1; } > $O/lite_ostage.log 2>&1 || { tail -20 $O/lite_ostage.log; exit 1; }
grep -E "==|expand| us |MISMATCH" $O/lite_ostage.log | grep -v "check: max |err| / sum|terms| = [0-9.]*e-0[78]$"
TAG=r9 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_ACC_NSLOT_X6=2@RST_ACC_NSLOT_X6=4@2 ab=RST_ACC_NSLOT_X6=1@RST_ACC_NSLOT_X6=4@2
