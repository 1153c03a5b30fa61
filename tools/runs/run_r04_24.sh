# r04 call 24: accumulator copies re-checked on the final frame: narrow/last 4 vs 8, residual 2 vs 4
mkdir -p gpurun_out
TAG=r24 bash tools/gpu_measure.sh ab=RST_ACC_NSLOT=4@-@3 ab=RST_ACC_NSLOT_X6=2@-@3
