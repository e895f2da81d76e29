#!/bin/bash
# Literal helix vs PLANE on MI355X: batch and single cubes, plus a rocprofv3
# kernel-trace summary of the literal helix at 512 x 256^3.
# usage (GPU box): bash scripts/gpu_literal.sh TAG
set -o pipefail
TAG=${1:-lit}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BV="python tools/bench_variants.py --kernel plane --check"
timeout -k 10 300 $BV --n 512 --L 256 --rounds 3 --variants TSA_PENCIL_MODE=literal TSA_PENCIL_MODE=plane > $OUT/batch.jsonl 2>$OUT/err.log || exit 1
for L in 64 128 256; do
  for N in 1 4 16; do
    timeout -k 10 200 $BV --n $N --L $L --rounds 5 --variants TSA_PENCIL_MODE=literal TSA_PENCIL_MODE=plane >> $OUT/single.jsonl 2>>$OUT/err.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TSA_PENCIL_MODE=literal timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lit --output-format csv -- python tools/bench_variants.py --kernel plane --n 512 --L 256 --rounds 5 --variants TSA_PENCIL_MODE=literal > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/literal_kernel_stats.csv \;
cat $OUT/batch.jsonl $OUT/single.jsonl
