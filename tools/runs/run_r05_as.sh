#!/bin/bash
# round 5: host-side enqueue cost of the training step's pieces (tools/host_launch_probe.py)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_launch_probe.py > gpurun_out/host_launch_r05as.log 2>&1; rc=$?; cat gpurun_out/host_launch_r05as.log; exit $rc
