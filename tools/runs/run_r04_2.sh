# r04 call: GPU tests (all failures listed), standalone narrow-layer benches (f32 vs x6) and timelines,
# finer wino_x6 timeline, last/wino9 timelines, then smoke, A/B against HEAD's library, default bench
mkdir -p gpurun_out
O=gpurun_out
TAG=x6n PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests; trc=$?
{ echo "== f32"; timeout -k 10 120 ./tools/lite_bench 200 && echo "== x6" && timeout -k 10 120 ./tools/lite_bench_x6 200 && \
  echo "== f32 prof" && timeout -k 10 120 ./tools/lite_bench_prof 50 && echo "== x6 prof" && timeout -k 10 120 ./tools/lite_bench_x6prof 50; } > $O/lite_x6.log 2>&1 || { tail -20 $O/lite_x6.log; exit 1; }
cat $O/lite_x6.log
{ for pro in 1 3; do timeout -k 10 120 ./tools/wino_x6_bench_prof 1 128 $pro 0 0 0 0 0 1 || exit 1; done
  timeout -k 10 120 ./tools/wino_x6_bench_prof 1 32 0 0 0 0 0 0 2 || exit 1
  timeout -k 10 120 ./tools/last_bench_prof 50 && timeout -k 10 120 ./tools/wino9_x6_bench_prof 1; } > $O/timelines2.log 2>&1 || { tail -20 $O/timelines2.log; exit 1; }
cat $O/timelines2.log
[ $trc -eq 0 ] || exit 1
TAG=x6n bash tools/gpu_measure.sh smoke ab=RST_LIB=tools/librst_head.so@-@3 bench
