#!/bin/bash
# r06s: the config-4 step's phases on the device clock (tools/step_phases.py), default and with serial targets
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06s_default.log 2>&1 && cat gpurun_out/phases_r06s_default.log && \
RST_SERIAL_TARGETS=1 timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06s_serialtargets.log 2>&1 && cat gpurun_out/phases_r06s_serialtargets.log && \
timeout -k 10 300 python -u tools/step_phases.py 20 > gpurun_out/phases_r06s_default2.log 2>&1 && cat gpurun_out/phases_r06s_default2.log
