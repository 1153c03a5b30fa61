# r04 call 17: write-through of the residual convs' materialised input (RST_WT_STORES 15 vs 13), four more pairs
mkdir -p gpurun_out
TAG=r17 bash tools/gpu_measure.sh ab=RST_WT_STORES=15@-@4
