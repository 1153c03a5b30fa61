# r04 call 6: narrow layers with per-wave CIN partials (accumulator path, one LDS merge per flush) and the x6
# B-operand ring depth 3, vs round-4 commit c022231 (lite_bench_x6_old), standalone and checked; GPU tests;
# A/B of the library against c022231; default bench
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do for v in x6 x6bd3 x6_old; do echo "== $v"; timeout -k 10 120 ./tools/lite_bench_$v 200 || exit 1; done; done
  echo "== x6 prof"; timeout -k 10 120 ./tools/lite_bench_x6prof 50 || exit 1; } > $O/lite_stats.log 2>&1 || { tail -20 $O/lite_stats.log; exit 1; }
grep -E "==|  us |MISMATCH" $O/lite_stats.log | grep -v check
TAG=r6 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_LIB=tools/librst_r4c.so@-@3 bench
