#!/bin/bash
# Same-box A/B of library builds on single cubes (lap kernel): 256^3 and 1024^3 (16-bit words).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for which in cur ${LIBS}; do
    if [ $which = cur ]; then unset TSA_PKG_DIR; else export TSA_PKG_DIR=$GRAFT_REPO_ROOT/scratch/$which; fi
    timeout -k 10 300 python tools/bench_variants.py --n 1 --L 256 --rounds 7 --variants "TSA_LAP_ZT=128" > gpurun_out/s256_$which.json 2>/dev/null || exit 1
    timeout -k 10 300 python tools/bench_variants.py --n 1 --L 1024 --rounds 3 --score-bits 16 --variants "TSA_LAP_ZT=128" > gpurun_out/s1024_$which.json 2>/dev/null || exit 1
    echo "$which 256: $(cut -c1-200 gpurun_out/s256_$which.json)"
    echo "$which 1024: $(cut -c1-200 gpurun_out/s1024_$which.json)"
  done
done
