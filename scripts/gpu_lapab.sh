#!/bin/bash
# Same-box A/B of lap-kernel build variants (scratch/<name> packages from
# scripts/build_variant.sh) on single cubes, interleaved over two repetitions.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V1="TSA_PENCIL_MODE=lap,TSA_LAP_M=1,TSA_LAP_NW=8 TSA_PENCIL_MODE=lap,TSA_LAP_M=1,TSA_LAP_NW=4"
for rep in 1 2; do
  for which in cur ${LIBS}; do
    if [ $which = cur ]; then unset TSA_PKG_DIR; else export TSA_PKG_DIR=$GRAFT_REPO_ROOT/scratch/$which; fi
    for L in ${SIZES:-64 256}; do
      timeout -k 10 200 python tools/bench_variants.py --n 1 --L $L --rounds 7 --check --variants $V1 \
        > gpurun_out/ab_${which}_$L.json 2> gpurun_out/ab_${which}_$L.err || { tail -5 gpurun_out/ab_${which}_$L.err; exit 1; }
      echo "$which L=$L"; cat gpurun_out/ab_${which}_$L.json
    done
  done
done
