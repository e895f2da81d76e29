#!/bin/bash
# Same-box A/B of the current library against scratch/oldpkg (a previous build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for which in new old; do
    if [ $which = old ]; then export TSA_PKG_DIR=$GRAFT_REPO_ROOT/scratch/oldpkg; else unset TSA_PKG_DIR; fi
    timeout -k 10 300 python tools/bench_variants.py --n 512 --rounds 5 --variants ${VARIANTS:-TSA_PENCIL_NW=8} > gpurun_out/ab_$which.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || exit $rc
    echo "$which: $(cat gpurun_out/ab_$which.json)"
  done
done
