# r04 call 20: narrow layers' prologue affine formed before (tf) or after the first tile's input loads, with the
# frame's accumulator-formed prologue (LITE_PROACC 4 / 8), alternating
mkdir -p gpurun_out
O=gpurun_out
{ for i in 1 2; do for n in 4 8; do for v in x6 x6tf; do echo "== $v proacc $n"; LITE_PROACC=$n timeout -k 10 120 ./tools/lite_bench_$v 200 || exit 1; done; done; done; } > $O/lite_tf.log 2>&1 || { tail -20 $O/lite_tf.log; exit 1; }
grep -E "==|expand.* us " $O/lite_tf.log
