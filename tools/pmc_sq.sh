#!/bin/bash
# SQ-counter passes (MFMA busy, wave stall breakdown, LDS) of the inference frame (tools/wino_probe.py) and of
# the training step (tools/train_step_run.py), one rocprofv3 --pmc pass per counter group, each under its own
# time limit (at most 8 SQ + 2 GRBM counters per pass, MI355X_MICROARCH.md §rocprofv3 PMC slots).
# Usage (GPU box, repo root): bash tools/pmc_sq.sh <tag> [frame|train]...   -> gpurun_out/sq_<tag>_<what>_<pass>/
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
whats=("$@"); [ ${#whats[@]} -eq 0 ] && whats=(frame)
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"
B="SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
for what in "${whats[@]}"; do
    case $what in
        frame) cmd=(python3 tools/wino_probe.py winograd_bf16x6 3) ;;
        train) cmd=(python3 tools/train_step_run.py --steps 1 --transfer winograd_bf16x6) ;;
        *) echo "unknown $what"; exit 2 ;;
    esac
    for p in A B; do
        d=gpurun_out/sq_${tag}_${what}_$p
        rm -rf "$d"
        timeout -s KILL 150 rocprofv3 --pmc ${!p} --output-format csv -d "$d" -o run -- "${cmd[@]}" \
            > "$d.log" 2>&1 || { tail -20 "$d.log"; exit 1; }
        echo "$what pass $p ok"
    done
done
