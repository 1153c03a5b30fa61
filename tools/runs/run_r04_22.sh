# r04 call 22: final tree: GPU tests, smoke, default bench
mkdir -p gpurun_out
TAG=r22 PYTEST_X=--maxfail=15 bash tools/gpu_measure.sh tests smoke bench
