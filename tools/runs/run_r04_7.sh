# r04 call 7: accumulator copies of the narrow / last layers (RST_ACC_NSLOT 8 and 4 vs the default 32), same box;
# frame kernel-trace profile
mkdir -p gpurun_out
TAG=r7 bash tools/gpu_measure.sh ab=RST_ACC_NSLOT=8@-@3 ab=RST_ACC_NSLOT=4@RST_ACC_NSLOT=16@2 prof
