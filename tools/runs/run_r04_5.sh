# r04 call 5: pipelined expand_0 x6 with unconditional loads (exact vmcnt across steps) vs round-4 HEAD's
# single-buffer form, standalone and checked; GPU tests; A/B of the library against the round-4 commit c022231
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do echo "== x6 pipe"; timeout -k 10 120 ./tools/lite_bench_x6 200 || exit 1
    echo "== x6 old"; timeout -k 10 120 ./tools/lite_bench_x6_old 200 || exit 1; done
  echo "== x6 pipe prof"; timeout -k 10 120 ./tools/lite_bench_x6prof 50 || exit 1; } > $O/lite_pipe2.log 2>&1 || { tail -20 $O/lite_pipe2.log; exit 1; }
grep -E "==|expand_0|MISMATCH" $O/lite_pipe2.log
TAG=r5 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_LIB=tools/librst_r4c.so@-@4
