# r04 first measurement call: dot2 split check, conv_lite per-CU sweep, per-kernel timelines, HEAD vs new tests, A/B, bench
mkdir -p gpurun_out
timeout -k 10 120 ./tools/dot2_split_check > gpurun_out/dot2_check.log 2>&1; cat gpurun_out/dot2_check.log
for n in 8 4 3 2 1; do echo "== per_cu $n"; RST_LITE_PER_CU=$n timeout -k 10 120 ./tools/lite_bench 200 || exit 1; done > gpurun_out/lite_percu.log 2>&1
cat gpurun_out/lite_percu.log
{ timeout -k 10 120 ./tools/wino_x6_bench_prof 1 128 1 0 0 0 0 0 1 && timeout -k 10 120 ./tools/last_bench_prof 50 && \
  timeout -k 10 120 ./tools/wino9_x6_bench_prof 1 && timeout -k 10 120 ./tools/lite_bench_prof 50; } > gpurun_out/timelines.log 2>&1 || exit 1
cat gpurun_out/timelines.log
TAG=head RST_LIB=tools/librst_head.so bash tools/gpu_measure.sh tests && TAG=d2 bash tools/gpu_measure.sh tests smoke ab=RST_LIB=tools/librst_head.so@-@3 bench
