#!/bin/bash
# The one GPU-box runner (run via gpurun from the repo root). Every GPU step has its own time limit; the steps are
# chained so the first failure ends the call (no retries). Outputs go to gpurun_out/<step>_<TAG>.* (TAG env, default "x").
#
# Usage: bash tools/gpu_measure.sh STEP...
#   tests[=K]        pytest -m gpu (optionally -k K; PYTEST_X overrides -x) -> pytest_<TAG>.log
#   smoke            __graft_entry__.smoke()                              -> smoke_<TAG>.log
#   bench[=ARGS]     bench.py (default flags, or ARGS with ',' for ' ')   -> bench_<TAG>.log
#   short            bench.py headline only (no side legs)                -> bench_short_<TAG>.log
#   prof             rocprofv3 --kernel-trace --stats of the short bench  -> prof_<TAG>/
#   trainprof        rocprofv3 --kernel-trace --stats of the training step -> trainprof_<TAG>/
#   trainhip         rocprofv3 --kernel-trace --hip-runtime-trace of the training step -> trainhip_<TAG>/
#   pmc              FETCH_SIZE / WRITE_SIZE passes of the frame probe    -> pmc_{f,w}_<TAG>/
#   sq[=frame|train] the SQ counter passes (tools/pmc_sq.sh)              -> sq_<TAG>_<what>_{A,B}/
#   ab=ENV_A@ENV_B@N alternating headline runs with env A then env B, N pairs ("-" = no env, ':' separates vars)
#   trainab=ENV_A@ENV_B@N the same for the config-4 training step
#   x6bench=ARGS     tools/wino_x6_bench ARGS (',' for ' ')               -> x6bench_<TAG>.log (appended)
#   x6prof=ARGS      tools/wino_x6_bench_prof ARGS (X6_PROF timeline)     -> x6prof_<TAG>.log
#   w9bench=ARGS     tools/wino9_x6_bench ARGS                            -> w9bench_<TAG>.log
#   litebench=ARGS   tools/lite_bench_x6 ARGS                             -> litebench_<TAG>.log
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-x}
O=gpurun_out
SHORT="--steps 100 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-batch 0"
TRAIN="--steps 5 --warmup 2 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor --no-ingest --pcie-steps 0 --no-two-styles --train-modes bf16 --train-steps 12"

fps() { grep -o '"value": [0-9.]*' "$1" | head -1 | grep -o '[0-9.]*$'; }
trainms() { grep -o '"training": {.\{0,420\}' "$1" | grep -o '"ms_per_step": [0-9.]*' | grep -o '[0-9.]*$'; }
runenv() {  # runenv "A=1:B=2" cmd...
    local e=$1; shift
    if [ "$e" = "-" ]; then "$@"; else env $(echo "$e" | tr ':' ' ') "$@"; fi
}

for step in "$@"; do
    name=${step%%=*}; arg=""; [ "$name" != "$step" ] && arg=${step#*=}
    case $name in
    tests)
        k=(); [ -n "$arg" ] && k=(-k "$arg")
        timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X:--x} -v --timeout 300 --timeout-method thread "${k[@]}" \
            > $O/pytest_$TAG.log 2>&1 || { tail -40 $O/pytest_$TAG.log; exit 1; }
        tail -1 $O/pytest_$TAG.log ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 \
            || { tail -30 $O/smoke_$TAG.log; exit 1; }
        tail -2 $O/smoke_$TAG.log ;;
    bench)
        timeout -k 10 900 python -u bench.py ${arg//,/ } > $O/bench_$TAG.log 2>&1 || { tail -30 $O/bench_$TAG.log; exit 1; }
        echo "bench: $(fps $O/bench_$TAG.log) FPS, training $(trainms $O/bench_$TAG.log) ms" ;;
    short)
        timeout -k 10 300 python -u bench.py $SHORT > $O/bench_short_$TAG.log 2>&1 || { tail -30 $O/bench_short_$TAG.log; exit 1; }
        echo "short: $(fps $O/bench_short_$TAG.log) FPS" ;;
    prof)
        rm -rf $O/prof_$TAG
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- \
            python bench.py --steps 50 --warmup 10 --no-cpu-baseline --stream-batch 0 --no-bf16x3 --no-predictor \
            --no-ingest --pcie-steps 0 --train-batch 0 --no-two-styles > $O/prof_$TAG.log 2>&1 || { tail -30 $O/prof_$TAG.log; exit 1; }
        echo "prof ok" ;;
    trainprof)
        rm -rf $O/trainprof_$TAG
        timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trainprof_$TAG -o run -- \
            python bench.py $TRAIN > $O/trainprof_$TAG.log 2>&1 || { tail -30 $O/trainprof_$TAG.log; exit 1; }
        echo "trainprof ok" ;;
    trainhip)   # kernel + HIP runtime API trace of the training step (host issue vs device time)
        rm -rf $O/trainhip_$TAG
        timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/trainhip_$TAG -o run -- \
            python bench.py $TRAIN > $O/trainhip_$TAG.log 2>&1 || { tail -30 $O/trainhip_$TAG.log; exit 1; }
        echo "trainhip ok" ;;
    pmc)
        rm -rf $O/pmc_f_$TAG $O/pmc_w_$TAG
        timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f_$TAG -o run -- \
            python tools/wino_probe.py winograd_bf16x6 3 > $O/pmc_f_$TAG.log 2>&1 || { tail -20 $O/pmc_f_$TAG.log; exit 1; }
        timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w_$TAG -o run -- \
            python tools/wino_probe.py winograd_bf16x6 3 > $O/pmc_w_$TAG.log 2>&1 || { tail -20 $O/pmc_w_$TAG.log; exit 1; }
        echo "pmc ok" ;;
    sq)
        bash tools/pmc_sq.sh "$TAG" ${arg:-frame} || exit 1 ;;
    ab|trainab)
        IFS=@ read -r ea eb n <<< "$arg"
        for i in $(seq 1 ${n:-3}); do
            for side in a b; do
                e=$ea; [ $side = b ] && e=$eb
                f=$O/${name}_${TAG}_${side}_$i.log
                if [ $name = ab ]; then
                    runenv "$e" timeout -k 10 300 python -u bench.py $SHORT > $f 2>&1 || { tail -30 $f; exit 1; }
                    echo "$name $side ($e) run $i: $(fps $f) FPS"
                else
                    runenv "$e" timeout -k 10 400 python -u bench.py $TRAIN > $f 2>&1 || { tail -30 $f; exit 1; }
                    echo "$name $side ($e) run $i: $(trainms $f) ms"
                fi
            done
        done ;;
    x6bench|x6prof|w9bench|w9prof|litebench)
        case $name in x6bench) b=tools/wino_x6_bench ;; x6prof) b=tools/wino_x6_bench_prof ;; w9bench) b=tools/wino9_x6_bench ;;
                      w9prof) b=tools/wino9_x6_bench_prof ;; litebench) b=tools/lite_bench_x6 ;; esac
        # several runs of one tool under one TAG append to its log
        echo "== $b ${arg//,/ }" >> $O/${name}_$TAG.log
        timeout -k 10 300 $b ${arg//,/ } >> $O/${name}_$TAG.log 2>&1 || { tail -30 $O/${name}_$TAG.log; exit 1; }
        tail -6 $O/${name}_$TAG.log ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
done
