# r04 call 10: x6 strided convs' output staged through LDS (contract_0 / _1) vs per-accumulator stores, standalone
# and checked; GPU tests; smoke; A/B of the library against round-4 commit c022231; default bench; frame
# kernel-trace profile and the FETCH/WRITE passes
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do for v in x6 x6nost0; do echo "== $v"; timeout -k 10 120 ./tools/lite_bench_$v 200 || exit 1; done; done
  echo "== x6prof"; timeout -k 10 120 ./tools/lite_bench_x6prof 50 || exit 1; } > $O/lite_ostage0.log 2>&1 || { tail -20 $O/lite_ostage0.log; exit 1; }
grep -E "==|contract| us |MISMATCH" $O/lite_ostage0.log | grep -v "check: max |err| / sum|terms| = [0-9.]*e-0[78]$"
TAG=r10 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests smoke ab=RST_LIB=tools/librst_r4c.so@-@3 bench prof pmc
