#!/bin/bash
# round 5: kernel trace of the standalone start-conv bench (the F3 full-block launch and the half-unit tail launch)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/f3prof_r05h
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f3prof_r05h -o run -- tools/wino9f3_bench 1 > gpurun_out/f3prof_r05h.log 2>&1 || { tail -20 gpurun_out/f3prof_r05h.log; exit 1; }
cat gpurun_out/f3prof_r05h/run_kernel_stats.csv | cut -d, -f1-4
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/f3prof_r05h/run_kernel_trace.csv')) if 'wino9f3' in r['Kernel_Name']]
ts=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'][:40]) for r in rows]
ts.sort()
for a,b,n in ts[10:16]: print(n, (b-a)/1000, 'us, gap to next', )
for i in range(10,16): print('gap', (ts[i+1][0]-ts[i][1])/1000)
PY
