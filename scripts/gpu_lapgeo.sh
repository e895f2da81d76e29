#!/bin/bash
# Lap geometry sweep on large single cubes (same box, spin preload): every
# (M, NW) the planner may pick, 16-bit words, plus the checked kernel's pick
# at the RTL's 12-bit words. Results: gpurun_out/$TAG/lapgeo.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-lapgeo}; O=gpurun_out/$TAG; mkdir -p $O
run() { echo "== $*" >> $O/lapgeo.jsonl; timeout -k 10 300 python tools/bench_variants.py "$@" >> $O/lapgeo.jsonl 2>> $O/lapgeo.err; }
for L in ${LENS:-1024 768}; do
  run --n 1 --L $L --rounds 5 --score-bits 16 --preload --variants "TSA_NONE=0" \
    "TSA_PENCIL_MODE=lap,TSA_LAP_M=1,TSA_LAP_NW=8" "TSA_PENCIL_MODE=lap,TSA_LAP_M=2,TSA_LAP_NW=8" "TSA_PENCIL_MODE=lap,TSA_LAP_M=4,TSA_LAP_NW=8" "TSA_PENCIL_MODE=lap,TSA_LAP_M=4,TSA_LAP_NW=4" || exit 1
done
run --n 1 --L 1024 --rounds 5 --kernel checked --preload --variants "TSA_NONE=0" "TSA_PENCIL_MODE=lap,TSA_LAP_M=1,TSA_LAP_NW=8" || exit 1
cat $O/lapgeo.jsonl
