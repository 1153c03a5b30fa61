# r04 call 28: x6 start-conv weight gradient with a bank-conflict-free channel pitch: training parity tests with it on,
# then the config-4 step on (RST_WGRAD9_X6=1) vs off, same box
mkdir -p gpurun_out
RST_WGRAD9_X6=1 TAG=r28 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests=train && TAG=r28 bash tools/gpu_measure.sh trainab=RST_WGRAD9_X6=1@-@2
