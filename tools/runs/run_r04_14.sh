# r04 call 14: residual convs' one-barrier per-wave statistics (accumulator path) vs c022231's two-pass tile form,
# standalone (wino_x6_bench, producer + consumer accumulators), alternating; GPU tests; library A/B vs c022231
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2 3; do for v in wino_x6_bench wino_x6_bench_old; do for p in 1 3; do echo "== $v pro $p"
      timeout -k 10 120 ./tools/$v 1 128 $p 0 0 0 0 0 1 || exit 1; done; done; done; } > $O/x6_stats.log 2>&1 || { tail -20 $O/x6_stats.log; exit 1; }
grep -E "==|us/launch|max" $O/x6_stats.log | head -60
# narrow layers with the prologue affine formed from producer accumulators (as in the frame) vs given
{ for i in 1 2; do echo "== given"; timeout -k 10 120 ./tools/lite_bench_x6 200 || exit 1
    echo "== proacc 4"; LITE_PROACC=4 timeout -k 10 120 ./tools/lite_bench_x6 200 || exit 1
    echo "== proacc 8"; LITE_PROACC=8 timeout -k 10 120 ./tools/lite_bench_x6 200 || exit 1; done
  echo "== proacc 4 prof"; LITE_PROACC=4 timeout -k 10 120 ./tools/lite_bench_x6prof 50 || exit 1; } > $O/lite_proacc.log 2>&1 || { tail -20 $O/lite_proacc.log; exit 1; }
grep -E "==|expand.* us " $O/lite_proacc.log
TAG=r14 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_LIB=tools/librst_r4c.so@-@2
