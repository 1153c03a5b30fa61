# r04 call 12: bank-conflict-free staging thread map for the x6 transposed convs vs quad-fastest, standalone and
# checked; GPU tests; SQ passes of the frame (LDS bank conflicts)
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do for v in x6 x6noremap; do echo "== $v"; timeout -k 10 120 ./tools/lite_bench_$v 200 || exit 1; done; done; } > $O/lite_remap.log 2>&1 || { tail -20 $O/lite_remap.log; exit 1; }
grep -E "==| us |MISMATCH" $O/lite_remap.log | grep -v "check: max |err| / sum|terms| = [0-9.]*e-0[78]$"
TAG=r12 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests sq
