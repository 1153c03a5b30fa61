# r04 call 21: narrow layers' prologue affine before the first tile's loads (LITE_TABLE_FIRST 1) in the frame vs commit
# 510b30e (same box); GPU tests
mkdir -p gpurun_out
TAG=r21 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests ab=RST_LIB=tools/librst_r4e.so@-@4
