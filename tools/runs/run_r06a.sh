#!/bin/bash
# r06a: probes (graph event timing, FETCH/WRITE calibration, in-launch barrier) + HEAD baseline short bench / rocprof
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 120 ./tools/probe_r06 graphev 1000 > $O/graphev.log 2>&1 && cat $O/graphev.log &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/graphev_prof -o run -- ./tools/probe_r06 graphev 1000 > $O/graphev_prof.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_f -o run -- ./tools/probe_r06 fetch > $O/fetch_f.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/fetch_w -o run -- ./tools/probe_r06 fetch > $O/fetch_w.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d $O/fetch_r -o run -- ./tools/probe_r06 fetch > $O/fetch_r.log 2>&1 &&
timeout -k 10 120 ./tools/probe_r06 barrier 1000 > $O/barrier.log 2>&1 && cat $O/barrier.log &&
TAG=r06a bash tools/gpu_measure.sh short prof
