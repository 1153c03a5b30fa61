# r04 call 16: write-through store bits re-checked on the round-4 frame (15: + wino_x6 materialised input; 9: wino9_x6
# output plain) vs the default 13
mkdir -p gpurun_out
TAG=r16 bash tools/gpu_measure.sh ab=RST_WT_STORES=15@-@3 ab=RST_WT_STORES=9@-@3
