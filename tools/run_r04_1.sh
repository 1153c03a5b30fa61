mkdir -p gpurun_out
timeout -k 10 120 ./tools/dot2_split_check > gpurun_out/dot2_check.log 2>&1; cat gpurun_out/dot2_check.log
for n in 8 4 3 2 1; do echo "== per_cu $n"; RST_LITE_PER_CU=$n timeout -k 10 120 ./tools/lite_bench 200 || exit 1; done > gpurun_out/lite_percu.log 2>&1
cat gpurun_out/lite_percu.log
TAG=head RST_LIB=tools/librst_head.so bash tools/gpu_measure.sh tests && TAG=d2 bash tools/gpu_measure.sh tests smoke ab=RST_LIB=tools/librst_head.so@-@3 bench
