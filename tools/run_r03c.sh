#!/bin/bash
# r03 measurement pass, part 2: residual / start-conv standalone benches before and after this round's
# changes, SQ-counter passes (standalone residual kernel, frame, training step), rocprofv3 kernel stats of
# the frame loop, and the no-SLP narrow/last-conv library variant. Each GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/x6b.log gpurun_out/w9b.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_transfer.py -x -v --timeout 200 --timeout-method thread -k "two_style" \
    > gpurun_out/pytest_s2.log 2>&1 || { tail -30 gpurun_out/pytest_s2.log; exit 1; }
tail -2 gpurun_out/pytest_s2.log
for b in wino_x6_bench wino_x6_bench_v2; do
    for args in "1 128 1 0 0 0 0 1" "1 128 1" "1 128 3" "1 128 2"; do
        echo "== $b $args" >> gpurun_out/x6b.log
        timeout -k 5 60 tools/$b $args >> gpurun_out/x6b.log 2>&1 || { tail -20 gpurun_out/x6b.log; exit 1; }
    done
done
grep "==\|wino_x6 B" gpurun_out/x6b.log
for b in wino9_x6_bench_v1 wino9_x6_bench_v2; do
    echo "== $b" >> gpurun_out/w9b.log
    timeout -k 5 60 tools/$b 1 >> gpurun_out/w9b.log 2>&1 || { tail -20 gpurun_out/w9b.log; exit 1; }
done
cat gpurun_out/w9b.log
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for b in wino_x6_bench wino_x6_bench_v2; do
    for p in A B; do
        d=gpurun_out/sq_${b}_$p; rm -rf $d
        timeout -s KILL 60 rocprofv3 --pmc ${!p} --output-format csv -d $d -o run -- tools/$b 1 128 3 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    done
done
echo "x6 pmc ok"
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 \
    --no-predictor --train-batch 0 --no-ingest --no-two-styles --pcie-steps 0 > gpurun_out/bench_base.log 2>&1 || { tail -30 gpurun_out/bench_base.log; exit 1; }
RST_LIB=tools/librst_noslp.so timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --stream-batch 0 \
    --no-bf16x3 --no-predictor --train-batch 0 --no-ingest --no-two-styles --pcie-steps 0 > gpurun_out/bench_noslp.log 2>&1 || { tail -30 gpurun_out/bench_noslp.log; exit 1; }
echo "noslp ok"
bash tools/pmc_sq.sh v2 frame train || exit 1
rm -rf gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 50 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor \
    --train-batch 0 --no-ingest --no-two-styles --pcie-steps 0 > gpurun_out/bench_prof.log 2>&1 || { tail -30 gpurun_out/bench_prof.log; exit 1; }
echo "prof ok"
