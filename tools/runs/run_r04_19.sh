# r04 call 19: output kernel with its input loads ahead of the affine merge vs commit 510b30e (same box); next-layer
# L2 touches off (RST_NO_U_PREFETCH=1) vs on, re-checked on the round-4 frame; GPU tests
mkdir -p gpurun_out
TAG=r19 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_LIB=tools/librst_r4e.so@-@3 ab=RST_NO_U_PREFETCH=1@-@2 prof
