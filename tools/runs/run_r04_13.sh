# r04 call 13: final-code measurement: GPU tests, smoke, default bench, frame kernel trace, A/B vs c022231
mkdir -p gpurun_out
TAG=r13 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests smoke bench prof ab=RST_LIB=tools/librst_r4c.so@-@2
