#!/bin/bash
# Same-box A/B of library builds: the in-tree package and each variants/<name>
# in $LIBS, interleaved, two repetitions (guide rule 24). Parity-checked.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
CHK=--check; [ -n "$NOCHECK" ] && CHK=""  # NOCHECK=1: timing-only experiment builds
for rep in 1 2; do
  for which in cur ${LIBS}; do
    if [ $which = cur ]; then unset TSA_PKG_DIR; else export TSA_PKG_DIR=$GRAFT_REPO_ROOT/variants/$which; fi
    timeout -k 10 300 python tools/bench_variants.py $CHK --n ${N:-512} --L ${L:-256} --rounds 5 \
      --variants ${VARIANTS:-TSA_PENCIL_NW=8} > gpurun_out/ab_$which.json 2> gpurun_out/ab_$which.err
    rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$which.err; exit $rc; }
    echo "$which: $(cat gpurun_out/ab_$which.json)"
  done
done
