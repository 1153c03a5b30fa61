#!/bin/bash
# r03 measurement pass (GPU box, repo root): two-style tests, bench, the residual kernel before/after the
# uniform-wave fix (standalone bench: timing + SQ passes), SQ passes of the frame and the training step,
# rocprofv3 kernel stats of the frame loop. Every GPU step has its own limit; the first failure ends the call.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transfer.py -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_transfer.log 2>&1 || { tail -30 gpurun_out/pytest_transfer.log; exit 1; }
tail -2 gpurun_out/pytest_transfer.log
timeout -k 10 420 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -c 400 gpurun_out/bench.log; echo
for b in wino_x6_bench wino_x6_bench_v2; do
    for args in "1 128 1 0 0 0 0 1" "1 128 1" "1 128 3" "1 128 2" "1 128 3 0 0 1 1"; do
        echo "== $b $args" >> gpurun_out/x6b.log
        timeout -k 5 60 tools/$b $args >> gpurun_out/x6b.log 2>&1 || { tail -20 gpurun_out/x6b.log; exit 1; }
    done
done
grep "wino_x6 B" gpurun_out/x6b.log
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for b in wino_x6_bench wino_x6_bench_v2; do
    for p in A B; do
        d=gpurun_out/sq_${b}_$p; rm -rf $d
        timeout -s KILL 60 rocprofv3 --pmc ${!p} --output-format csv -d $d -o run -- tools/$b 1 128 3 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    done
done
echo "x6 pmc ok"
bash tools/pmc_sq.sh v2 frame train || exit 1
rm -rf gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 50 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor \
    --train-batch 0 --no-ingest --no-two-styles --pcie-steps 0 > gpurun_out/bench_prof.log 2>&1 || { tail -30 gpurun_out/bench_prof.log; exit 1; }
echo "prof ok"
