#!/bin/bash
# Same-box A/B of library builds: the in-tree one ("cur") and scratch/<name> dirs
# (PKGS="name1 name2"), each in its own process; ARGS are bench_variants options.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do
  for which in cur ${PKGS}; do
    if [ $which = cur ]; then unset TSA_PKG_DIR; else export TSA_PKG_DIR=$GRAFT_REPO_ROOT/scratch/$which; fi
    timeout -k 10 300 python tools/bench_variants.py ${ARGS} > gpurun_out/pk_$which.json 2>/dev/null
    rc=$?; [ $rc -eq 0 ] || { echo "$which failed rc=$rc"; exit $rc; }
    echo "$which: $(cat gpurun_out/pk_$which.json | tr '\n' ' ')"
  done
done
