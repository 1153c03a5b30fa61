# r04 call 15: start conv with the self-resetting work queue (the last round's half units to the first finishers)
# vs the static unit order, standalone (checked against the f32 composite Winograd) and in the frame (same box)
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2 3; do echo "== static"; timeout -k 10 120 ./tools/wino9_x6_bench 1 || exit 1
    echo "== queue"; W9_QUEUE=1 timeout -k 10 120 ./tools/wino9_x6_bench 1 || exit 1; done
  echo "== queue prof"; W9_QUEUE=1 timeout -k 10 120 ./tools/wino9_x6_bench_prof 1 || exit 1; } > $O/w9_queue.log 2>&1 || { tail -20 $O/w9_queue.log; exit 1; }
grep -E "==|us/launch|max|grid span" $O/w9_queue.log
TAG=r15 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_W9_QUEUE=0@-@3
