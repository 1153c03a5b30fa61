# r04 call 8: same-box A/B of the narrow layers' write-through stores (RST_WT_STORES 5 = off for conv_lite) and of
# the residual convs' accumulator copies (RST_ACC_NSLOT_X6 4 vs 8); narrow-layer epilogue cost split (LITE_SKIP 8 =
# no output stores, 32 = no statistics)
mkdir -p gpurun_out
O=gpurun_out
{ for v in x6prof x6prof_s8 x6prof_s32; do echo "== $v"; timeout -k 10 120 ./tools/lite_bench_$v 50 || exit 1; done; } > $O/lite_epi.log 2>&1 || { tail -20 $O/lite_epi.log; exit 1; }
grep -E "==|per step| us " $O/lite_epi.log | grep -v check
TAG=r8 bash tools/gpu_measure.sh ab=RST_WT_STORES=5@-@3 ab=RST_ACC_NSLOT_X6=4@-@3
