# r04 call: GPU tests (all failures listed); wino_x6 accumulator-mode timelines (0 none, 1 both, 2 producer, 3 consumer);
# then smoke, A/B against HEAD's library, default bench
mkdir -p gpurun_out
O=gpurun_out
TAG=r3 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests; trc=$?
{ for m in 0 1 2 3; do timeout -k 10 120 ./tools/wino_x6_bench_prof 1 128 1 0 0 0 0 0 $m || exit 1; done
  for m in 0 1; do timeout -k 10 120 ./tools/wino_x6_bench 1 128 1 0 0 0 0 0 $m || exit 1; done
  echo "== affine first"; timeout -k 10 120 ./tools/wino_x6_bench_prof_af 1 128 1 0 0 0 0 0 1 || exit 1; } > $O/x6_accm.log 2>&1 || { tail -20 $O/x6_accm.log; exit 1; }
grep -E "timeline|us/launch" $O/x6_accm.log
timeout -k 10 120 ./tools/affine_probe > $O/affine_probe.log 2>&1 || { cat $O/affine_probe.log; exit 1; }
cat $O/affine_probe.log
# packed-f32 (SLP-vectorised) transforms vs scalar, standalone, alternating
{ for i in 1 2; do timeout -k 10 120 ./tools/wino9_x6_bench 1 && timeout -k 10 120 ./tools/wino9_x6_bench_slp 1 && \
  timeout -k 10 120 ./tools/wino_x6_bench 1 128 1 0 0 0 0 0 1 && timeout -k 10 120 ./tools/wino_x6_bench_slp 1 128 1 0 0 0 0 0 1 || exit 1; done; } > $O/slp_ab.log 2>&1 || { tail -20 $O/slp_ab.log; exit 1; }
grep -E "us/launch" $O/slp_ab.log
# start-conv wave stagger (W9_STAGGER s_sleep units), alternating
{ for i in 1 2; do for v in "" _st2 _st4 _st8 _pipe _pipeslp _slp; do echo "== w9$v"; timeout -k 10 120 ./tools/wino9_x6_bench$v 1 || exit 1; done; done; } > $O/w9_stagger.log 2>&1 || { tail -20 $O/w9_stagger.log; exit 1; }
grep -E "==|us/launch" $O/w9_stagger.log
[ $trc -eq 0 ] || exit 1
TAG=r3 bash tools/gpu_measure.sh smoke ab=RST_LIB=tools/librst_head.so@-@3 bench
