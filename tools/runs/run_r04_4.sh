# r04 call 4: pipelined expand_0 x6 (16-channel chunks, double-buffered LDS) vs round-4 HEAD's single-buffer form,
# standalone and checked (lite_bench sampled CPU check); then GPU tests, smoke, A/B vs round-3 HEAD, default bench,
# kernel-trace profile and the FETCH/WRITE passes
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do echo "== x6 pipe"; timeout -k 10 120 ./tools/lite_bench_x6 200 || exit 1
    echo "== x6 old"; timeout -k 10 120 ./tools/lite_bench_x6_old 200 || exit 1; done
  echo "== f32"; timeout -k 10 120 ./tools/lite_bench 200 || exit 1
  echo "== x6 pipe prof"; timeout -k 10 120 ./tools/lite_bench_x6prof 50 || exit 1; } > $O/lite_pipe.log 2>&1 || { tail -20 $O/lite_pipe.log; exit 1; }
grep -E "==|expand_0|MISMATCH" $O/lite_pipe.log
TAG=r4 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests smoke ab=RST_LIB=tools/librst_head.so@-@3 bench prof pmc
