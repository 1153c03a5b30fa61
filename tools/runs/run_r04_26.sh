# r04 call 26: start-conv weight gradient on split-bf16 x6 (x6 trainer): GPU tests (training parity included), then
# the config-4 training step with RST_WGRAD9_X6=0 (f32 kernel) vs the x6 kernel, same box
mkdir -p gpurun_out
TAG=r26 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests trainab=RST_WGRAD9_X6=0@-@2
