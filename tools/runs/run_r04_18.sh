# r04 call 18: end-of-session measurement: GPU tests, smoke, default bench, frame kernel trace, FETCH/WRITE passes,
# A/B vs c022231
mkdir -p gpurun_out
TAG=r18 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests smoke bench prof pmc ab=RST_LIB=tools/librst_r4c.so@-@3
